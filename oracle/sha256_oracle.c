/*
 * oracle/sha256_oracle.c -- CPU restatement of the reference hash path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity CHECKER: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product (mirbft_amd/libmirsha.so) never links, loads or falls back to it.
 *
 * What it restates
 * ----------------
 * 1. processor.ProcessHashActions  (/root/reference/pkg/processor/serial.go:180-198):
 *      for each action, in list order:
 *          h := hasher.New(); for _, d := range Hash.Data { h.Write(d) }; digest = h.Sum(nil)
 *    -> oracle_process_hash_actions(): parts are streamed through ONE running
 *       context per action (no concatenation buffer), exactly like h.Write.
 * 2. processor.Hasher = crypto.SHA256 (/root/reference/mirbft_test.go:392,
 *    /root/reference/pkg/testengine/recorder.go:781), i.e. the Go standard
 *    library crypto/sha256 of Go 1.15/1.16 (/root/reference/go.mod:3,
 *    /root/reference/.travis.yml:5-6). That package is NOT in /root/reference
 *    and no Go toolchain exists here, so its published algorithm -- FIPS 180-4
 *    section 6.2 (SHA-256) with the section 5.1.1 padding -- is restated below
 *    from the standard: digest.Write buffers to 64-byte blocks, digest.Sum pads
 *    with 0x80, zeros, and the 64-bit big-endian bit length.
 * 3. Client.Propose request digest (/root/reference/pkg/processor/clients.go:189-192)
 *    is the one-part case of (1).
 *
 * Pinning: tests/test_oracle.py checks this file against the FIPS 180-4 /
 * NIST known-answer vectors committed in tests/golden/kat.json and against an
 * independent implementation (Python hashlib = OpenSSL 3.0.2) on every golden
 * fixture. No reference test checks a digest directly.
 *
 * Deliberately plain scalar C: one context, one block at a time, no SIMD, so
 * that the CPU baseline it provides is the single-goroutine reference loop
 * (/root/reference/mirbft.go:470 runs hashing on one goroutine).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

typedef struct {
    uint32_t h[8];
    uint8_t buf[64];
    uint32_t nbuf;
    uint64_t len;
} oracle_sha256_ctx;

static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

/* FIPS 180-4 6.2.2: one compression of a 64-byte block. */
static void oracle_block(uint32_t h[8], const uint8_t* p) {
    uint32_t w[64];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) |
               ((uint32_t)p[4 * t + 2] << 8) | (uint32_t)p[4 * t + 3];
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = s1 + w[t - 7] + s0 + w[t - 16];
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 64; ++t) {
        uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t T1 = hh + S1 + ch + K256[t] + w[t];
        uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
        uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t T2 = S0 + maj;
        hh = g; g = f; f = e; e = d + T1; d = c; c = b; b = a; a = T1 + T2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* hasher.New() */
void oracle_sha256_init(oracle_sha256_ctx* c) {
    static const uint32_t IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    memcpy(c->h, IV, sizeof IV);
    c->nbuf = 0;
    c->len = 0;
}

/* h.Write(p): buffer to whole blocks, as Go's digest.Write does. */
void oracle_sha256_write(oracle_sha256_ctx* c, const uint8_t* p, size_t n) {
    c->len += n;
    if (c->nbuf) {
        size_t take = 64 - c->nbuf < n ? 64 - c->nbuf : n;
        memcpy(c->buf + c->nbuf, p, take);
        c->nbuf += (uint32_t)take; p += take; n -= take;
        if (c->nbuf == 64) { oracle_block(c->h, c->buf); c->nbuf = 0; }
    }
    while (n >= 64) { oracle_block(c->h, p); p += 64; n -= 64; }
    if (n) { memcpy(c->buf, p, n); c->nbuf = (uint32_t)n; }
}

/* h.Sum(nil): pad a COPY (Go's Sum does not reset the running digest). */
void oracle_sha256_sum(const oracle_sha256_ctx* c0, uint8_t out[32]) {
    oracle_sha256_ctx c = *c0;
    uint64_t bits = c.len * 8;
    uint8_t pad[72] = {0x80};
    size_t padlen = (c.len % 64 < 56) ? 56 - c.len % 64 : 120 - c.len % 64;
    for (int i = 0; i < 8; ++i) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
    oracle_sha256_write(&c, pad, padlen + 8);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(c.h[i] >> 24); out[4 * i + 1] = (uint8_t)(c.h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c.h[i] >> 8); out[4 * i + 3] = (uint8_t)c.h[i];
    }
}

void oracle_sha256(const uint8_t* p, uint64_t n, uint8_t out[32]) {
    oracle_sha256_ctx c;
    oracle_sha256_init(&c);
    oracle_sha256_write(&c, p, (size_t)n);
    oracle_sha256_sum(&c, out);
}

/*
 * ProcessHashActions (serial.go:180-198) over a packed arena: action i owns
 * parts [part_begin[i], part_begin[i+1]); part j is arena[part_off[j] : +part_len[j]].
 * Zero parts -> SHA256(""); empty parts contribute nothing. Output i*32.
 */
void oracle_process_hash_actions(const uint8_t* arena, const uint64_t* part_off,
                                 const uint64_t* part_len, const uint64_t* part_begin,
                                 uint64_t n_actions, uint8_t* out) {
    for (uint64_t i = 0; i < n_actions; ++i) {
        oracle_sha256_ctx c;
        oracle_sha256_init(&c);
        for (uint64_t j = part_begin[i]; j < part_begin[i + 1]; ++j)
            oracle_sha256_write(&c, arena + part_off[j], (size_t)part_len[j]);
        oracle_sha256_sum(&c, out + 32 * i);
    }
}

/* One-part actions (request digests, clients.go:189-192): message i = arena[off[i] : +len[i]]. */
void oracle_digest_batch(const uint8_t* arena, const uint64_t* off, const uint64_t* len,
                         uint64_t n, uint8_t* out) {
    for (uint64_t i = 0; i < n; ++i) oracle_sha256(arena + off[i], len[i], out + 32 * i);
}

/* Batch digest over request-ack digests (sequence.go:155-158): SHA256(concat(table[idx[k]])). */
void oracle_digest_of_digests(const uint8_t* table, const uint32_t* idx, const uint64_t* begin,
                              uint64_t n, uint8_t* out) {
    for (uint64_t i = 0; i < n; ++i) {
        oracle_sha256_ctx c;
        oracle_sha256_init(&c);
        for (uint64_t k = begin[i]; k < begin[i + 1]; ++k)
            oracle_sha256_write(&c, table + 32 * (uint64_t)idx[k], 32);
        oracle_sha256_sum(&c, out + 32 * i);
    }
}
