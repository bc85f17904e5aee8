/*
 * Second CPU oracle -- TEST INFRASTRUCTURE ONLY (see oracle.py): the loop of
 * processor.ProcessHashActions (/root/reference/pkg/processor/serial.go:180-198)
 * for one-part messages, each digest computed by OpenSSL libcrypto
 * (EVP_Digest{Init,Update,Final}, SHA-256; SHA-NI on CPUs that have it), split over
 * T POSIX threads in contiguous ranges. It cross-checks sha256_oracle.c and is
 * bench.py's strongest CPU baseline (the reference's own Go crypto/sha256
 * cannot be built in this image).
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>

struct range {
  const uint8_t* arena;
  const uint64_t* off;
  const uint64_t* len;
  uint64_t lo, hi;
  uint8_t* out;
  int rc;
};

static void* run_range(void* arg) {
  struct range* r = (struct range*)arg;
  /* explicitly fetched once per thread: EVP_sha256() would re-fetch (under a
   * global provider lock) on every init, serialising the threads */
  EVP_MD* md = EVP_MD_fetch(NULL, "SHA256", NULL);
  EVP_MD_CTX* c = EVP_MD_CTX_new();  /* one context per thread, reused per message */
  if (!c || !md) {
    EVP_MD_CTX_free(c);
    EVP_MD_free(md);
    r->rc = 1;
    return NULL;
  }
  for (uint64_t i = r->lo; i < r->hi; ++i) {
    unsigned int n = 32;
    if (!EVP_DigestInit_ex(c, md, NULL) || !EVP_DigestUpdate(c, r->arena + r->off[i], (size_t)r->len[i]) ||
        !EVP_DigestFinal_ex(c, r->out + 32 * i, &n) || n != 32) {
      r->rc = 1;
      break;
    }
  }
  EVP_MD_CTX_free(c);
  EVP_MD_free(md);
  return NULL;
}

/* out[32*i] = SHA-256(arena[off[i] : off[i]+len[i]]), i < n, over `threads`
 * threads (contiguous ranges). Returns 0 on success. */
int openssl_digest_batch(const uint8_t* arena, const uint64_t* off, const uint64_t* len, uint64_t n,
                         uint8_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if ((uint64_t)threads > n) threads = n ? (int)n : 1;
  struct range rs[256];
  pthread_t th[256];
  for (int t = 0; t < threads; ++t) {
    rs[t].arena = arena;
    rs[t].off = off;
    rs[t].len = len;
    rs[t].out = out;
    rs[t].rc = 0;
    rs[t].lo = n * (uint64_t)t / (uint64_t)threads;
    rs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
  }
  if (threads == 1) {
    run_range(&rs[0]);
    return rs[0].rc;
  }
  int started = 0;
  for (; started < threads; ++started)
    if (pthread_create(&th[started], NULL, run_range, &rs[started]) != 0) break;
  int rc = started == threads ? 0 : 1;
  for (int t = 0; t < started; ++t) {
    pthread_join(th[t], NULL);
    rc |= rs[t].rc;
  }
  return rc;
}
