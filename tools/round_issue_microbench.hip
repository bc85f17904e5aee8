// Issue cost of candidate two-lane SHA-256 round sequences on a lone wave
// (k_digest_chain2's consumer regime): each variant runs 16 rounds per asm
// statement, kIters statements, on one wave64 alone on its CU; s_memtime around
// the loop gives shader-clock ticks per round. Timing only (the variants that
// are not the shipped round compute nothing meaningful).
//   old11 : round 3/4's 11 instructions (2 row_mirror DPP)
//   new10 : 10 instructions, kh by an identity DPP (3 DPP)
//   new10v: new10 with the kh DPP replaced by a plain v_add (2 DPP)
//   valu11: 11 plain VALU, no DPP
//   dpp8  : 8 dependent-free identity DPP adds
//   valu8 : 8 plain independent v_add
//   new10b: new10 with the kh DPP before the first mirror DPP
//   new10u: new10 with the kh DPP unmasked (bank_mask 0xf)
//   old11+lds / old11+lds_e: old11 with a ds_read_b128 every 4 rounds (all lanes / e-lanes)
//   xad10+nop: kh by v_xad_u32 (no DPP), both mirror DPPs W = mirror(W) + u, s_nop 0 between
//   oct10 : round 5's candidate for VERDICT r4 #3, eight lanes a message -- each
//           lane ONE rotate (e-quad: 6/11/25, a-quad: 2/13/22), Sigma by two
//           quad_perm DPP xors, Ch and Maj, h + K+W, T1 by add3, T2, then e' and
//           a' by two DPP adds across the quads (row_ror:4 / row_ror:12, bank
//           masks): 10 instructions, 4 of them DPP
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/round_issue_microbench tools/round_issue_microbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int kIters = 2048;

#define R_OLD(X, Y, Z, W)                                                              \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"                             \
  "v_alignbit_b32 %[s2], %[" #X "], %[" #X "], %[sh2]\n\t"                             \
  "v_alignbit_b32 %[s3], %[" #X "], %[" #X "], %[sh3]\n\t"                             \
  "v_bitop3_b32 %[s], %[s1], %[s2], %[s3] bitop3:0x96\n\t"                            \
  "v_add_u32 %[sk], %[s], %[k]\n\t"                                                     \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                 \
  "v_add3_u32 %[u], %[sk], %[" #W "], %[c]\n\t"                                         \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t"                 \
  "v_add_u32 %[t], %[sk], %[m]\n\t"                                                     \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_mirror row_mask:0xf bank_mask:0x3\n\t" \
  "v_add_u32_dpp %[" #W "], %[u], %[t] row_mirror row_mask:0xf bank_mask:0xc\n\t"

#define R_NEW(X, Y, Z, W, KH)                                                          \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"                             \
  "v_alignbit_b32 %[s2], %[" #X "], %[" #X "], %[sh2]\n\t"                             \
  "v_alignbit_b32 %[s3], %[" #X "], %[" #X "], %[sh3]\n\t"                             \
  "v_bitop3_b32 %[s], %[s1], %[s2], %[s3] bitop3:0x96\n\t"                            \
  "v_bitop3_b32 %[c], %[M], %[" #X "], %[" #Y "] bitop3:0x9c\n\t"                      \
  "v_bitop3_b32 %[m], %[c], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                      \
  "v_add3_u32 %[u], %[s], %[kh], %[m]\n\t"                                              \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_mirror row_mask:0xf bank_mask:0x3\n\t" \
  KH                                                                                    \
  "v_add_u32_dpp %[" #W "], %[u], %[u] row_mirror row_mask:0xf bank_mask:0xc\n\t"

// new10 with the kh DPP between the add3 and the first mirror DPP
#define R_NEWB(X, Y, Z, W)                                                             \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"                             \
  "v_alignbit_b32 %[s2], %[" #X "], %[" #X "], %[sh2]\n\t"                             \
  "v_alignbit_b32 %[s3], %[" #X "], %[" #X "], %[sh3]\n\t"                             \
  "v_bitop3_b32 %[s], %[s1], %[s2], %[s3] bitop3:0x96\n\t"                            \
  "v_bitop3_b32 %[c], %[M], %[" #X "], %[" #Y "] bitop3:0x9c\n\t"                      \
  "v_bitop3_b32 %[m], %[c], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                      \
  "v_add3_u32 %[u], %[s], %[kh], %[m]\n\t"                                              \
  "v_add_u32_dpp %[kh], %[" #Z "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t" \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_mirror row_mask:0xf bank_mask:0x3\n\t" \
  "v_add_u32_dpp %[" #W "], %[u], %[u] row_mirror row_mask:0xf bank_mask:0xc\n\t"
// xad form: u' = (Z ^ M) + K' as the filler, then s_nop 0 before the a-lanes' DPP
#define R_XAD(X, Y, Z, W)                                                              \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"                             \
  "v_alignbit_b32 %[s2], %[" #X "], %[" #X "], %[sh2]\n\t"                             \
  "v_alignbit_b32 %[s3], %[" #X "], %[" #X "], %[sh3]\n\t"                             \
  "v_bitop3_b32 %[s], %[s1], %[s2], %[s3] bitop3:0x96\n\t"                            \
  "v_bitop3_b32 %[c], %[M], %[" #X "], %[" #Y "] bitop3:0x9c\n\t"                      \
  "v_bitop3_b32 %[m], %[c], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                      \
  "v_add3_u32 %[u], %[s], %[kh], %[m]\n\t"                                              \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_mirror row_mask:0xf bank_mask:0x3\n\t" \
  "v_xad_u32 %[kh], %[" #Z "], %[M], %[k]\n\t"                                          \
  "s_nop 0\n\t"                                                                        \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_mirror row_mask:0xf bank_mask:0xc\n\t"
#define R_OCT(X, Y, Z, W)                                                                  \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"                                 \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t"                     \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t"                     \
  "v_xor_b32_dpp %[s2], %[s1], %[s1] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"   \
  "v_add_u32 %[sk], %[" #W "], %[k]\n\t"                                                    \
  "v_xor_b32_dpp %[s], %[s1], %[s2] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"    \
  "v_add3_u32 %[u], %[s], %[c], %[sk]\n\t"                                                  \
  "v_add_u32 %[t], %[s], %[m]\n\t"                                                          \
  "v_add_u32_dpp %[" #W "], %[" #W "], %[u] row_ror:4 row_mask:0xf bank_mask:0x5\n\t"      \
  "v_add_u32_dpp %[" #W "], %[u], %[t] row_ror:12 row_mask:0xf bank_mask:0xa\n\t"
#define KH_DPPU(Z) "v_add_u32_dpp %[kh], %[" #Z "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0xf\n\t"
#define KH_DPP(Z) "v_add_u32_dpp %[kh], %[" #Z "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t"
#define KH_VALU(Z) "v_add_u32 %[kh], %[" #Z "], %[k]\n\t"

#define R_VALU11(X, Y, Z, W)                                           \
  "v_alignbit_b32 %[s1], %[" #X "], %[" #X "], %[sh1]\n\t"             \
  "v_alignbit_b32 %[s2], %[" #X "], %[" #X "], %[sh2]\n\t"             \
  "v_alignbit_b32 %[s3], %[" #X "], %[" #X "], %[sh3]\n\t"             \
  "v_bitop3_b32 %[s], %[s1], %[s2], %[s3] bitop3:0x96\n\t"            \
  "v_add_u32 %[sk], %[s], %[k]\n\t"                                     \
  "v_bitop3_b32 %[c], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xca\n\t" \
  "v_add3_u32 %[u], %[sk], %[" #W "], %[c]\n\t"                         \
  "v_bitop3_b32 %[m], %[" #X "], %[" #Y "], %[" #Z "] bitop3:0xe8\n\t" \
  "v_add_u32 %[t], %[sk], %[m]\n\t"                                     \
  "v_add_u32 %[" #W "], %[" #W "], %[u]\n\t"                            \
  "v_add_u32 %[" #W "], %[u], %[t]\n\t"

#define R_DPP8(X, Y, Z, W)                                                                   \
  "v_add_u32_dpp %[s1], %[" #X "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t" \
  "v_add_u32_dpp %[s2], %[" #Y "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t" \
  "v_add_u32_dpp %[s3], %[" #Z "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t" \
  "v_add_u32_dpp %[s], %[" #W "], %[k] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t"  \
  "v_add_u32_dpp %[c], %[" #X "], %[k] row_mirror row_mask:0xf bank_mask:0x3\n\t"           \
  "v_add_u32_dpp %[m], %[" #Y "], %[k] row_mirror row_mask:0xf bank_mask:0x3\n\t"           \
  "v_add_u32_dpp %[u], %[" #Z "], %[k] row_mirror row_mask:0xf bank_mask:0x3\n\t"           \
  "v_add_u32_dpp %[t], %[" #W "], %[k] row_mirror row_mask:0xf bank_mask:0x3\n\t"

#define R_VALU8(X, Y, Z, W)                       \
  "v_add_u32 %[s1], %[" #X "], %[k]\n\t"          \
  "v_add_u32 %[s2], %[" #Y "], %[k]\n\t"          \
  "v_add_u32 %[s3], %[" #Z "], %[k]\n\t"          \
  "v_add_u32 %[s], %[" #W "], %[k]\n\t"           \
  "v_add_u32 %[c], %[" #X "], %[k]\n\t"           \
  "v_add_u32 %[m], %[" #Y "], %[k]\n\t"           \
  "v_add_u32 %[u], %[" #Z "], %[k]\n\t"           \
  "v_add_u32 %[t], %[" #W "], %[k]\n\t"

// old11 with the consumer's LDS traffic: one ds_read_b128 of the next block's
// K+W every four rounds, by every lane (LDSA) or by the e-lanes only (LDSE: exec
// narrowed around the read, so the a-lanes' register keeps its 0)
#define LDSA "ds_read_b128 %[q], %[la]\n\t"
#define LDSE "s_mov_b64 exec, %[em]\n\t ds_read_b128 %[q], %[la]\n\t s_mov_b64 exec, -1\n\t"
#define FOURL(R, L) L R(X, Y, Z, W) R(W, X, Y, Z) R(Z, W, X, Y) R(Y, Z, W, X)
#define FOUR(R) R(X, Y, Z, W) R(W, X, Y, Z) R(Z, W, X, Y) R(Y, Z, W, X)
#define FOURN(KH) R_NEW(X, Y, Z, W, KH(Z)) R_NEW(W, X, Y, Z, KH(Y)) R_NEW(Z, W, X, Y, KH(X)) R_NEW(Y, Z, W, X, KH(W))

#define OPS                                                                                              \
  : [X] "+v"(X), [Y] "+v"(Y), [Z] "+v"(Z), [W] "+v"(W), [kh] "+v"(kh), [s1] "=&v"(s1), [s2] "=&v"(s2),   \
    [s3] "=&v"(s3), [s] "=&v"(s), [sk] "=&v"(sk), [c] "=&v"(c), [u] "=&v"(u), [m] "=&v"(m), [t] "=&v"(t) \
  : [sh1] "v"(sh1), [sh2] "v"(sh2), [sh3] "v"(sh3), [k] "v"(k), [M] "v"(M)

#define OPSL                                                                                             \
  : [X] "+v"(X), [Y] "+v"(Y), [Z] "+v"(Z), [W] "+v"(W), [s1] "=&v"(s1), [s2] "=&v"(s2),                \
    [s3] "=&v"(s3), [s] "=&v"(s), [sk] "=&v"(sk), [c] "=&v"(c), [u] "=&v"(u), [m] "=&v"(m), [t] "=&v"(t), \
    [q] "=&v"(q)                                                                                         \
  : [sh1] "v"(sh1), [sh2] "v"(sh2), [sh3] "v"(sh3), [k] "v"(k), [la] "v"(la), [em] "s"(em)               \
  : "memory"

template <int V>
__global__ __launch_bounds__(64) void k_rounds(uint32_t* out, uint64_t* ticks) {
  __shared__ uint4 lds[64 * 17];
  const unsigned lane = threadIdx.x;
  const bool eside = (lane & 15) < 8;
  uint32_t X = lane * 0x9E3779B9u, Y = X ^ 0x1234567u, Z = X + 77u, W = X * 3u, kh = 0;
  const uint32_t sh1 = eside ? 6 : 2, sh2 = eside ? 11 : 13, sh3 = eside ? 25 : 22, M = eside ? 0u : ~0u;
  const uint32_t k = lane * 0x85EBCA6Bu;
  uint32_t s1, s2, s3, s, sk, c, u, m, t;
  uint4 q = make_uint4(0, 0, 0, 0);
  lds[lane] = make_uint4(lane, 1, 2, 3);
  __syncthreads();
  const uint32_t la = (uint32_t)(uintptr_t)&lds[lane];
  const uint64_t em = 0x00ff00ff00ff00ffull;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
    if (V == 0) asm volatile(FOUR(R_OLD) FOUR(R_OLD) FOUR(R_OLD) FOUR(R_OLD) OPS);
    if (V == 1) asm volatile(FOURN(KH_DPP) FOURN(KH_DPP) FOURN(KH_DPP) FOURN(KH_DPP) OPS);
    if (V == 2) asm volatile(FOURN(KH_VALU) FOURN(KH_VALU) FOURN(KH_VALU) FOURN(KH_VALU) OPS);
    if (V == 3) asm volatile(FOUR(R_VALU11) FOUR(R_VALU11) FOUR(R_VALU11) FOUR(R_VALU11) OPS);
    if (V == 4) asm volatile(FOUR(R_DPP8) FOUR(R_DPP8) FOUR(R_DPP8) FOUR(R_DPP8) OPS);
    if (V == 5) asm volatile(FOUR(R_VALU8) FOUR(R_VALU8) FOUR(R_VALU8) FOUR(R_VALU8) OPS);
    if (V == 6) asm volatile(FOUR(R_NEWB) FOUR(R_NEWB) FOUR(R_NEWB) FOUR(R_NEWB) OPS);
    if (V == 7) asm volatile(FOURN(KH_DPPU) FOURN(KH_DPPU) FOURN(KH_DPPU) FOURN(KH_DPPU) OPS);
    if (V == 8) asm volatile(FOUR(R_XAD) FOUR(R_XAD) FOUR(R_XAD) FOUR(R_XAD) OPS);
    if (V == 9)
      asm volatile(FOURL(R_OLD, LDSA) FOURL(R_OLD, LDSA) FOURL(R_OLD, LDSA) FOURL(R_OLD, LDSA) "s_waitcnt lgkmcnt(0)\n\t" OPSL);
    if (V == 10)
      asm volatile(FOURL(R_OLD, LDSE) FOURL(R_OLD, LDSE) FOURL(R_OLD, LDSE) FOURL(R_OLD, LDSE) "s_waitcnt lgkmcnt(0)\n\t" OPSL);
    if (V == 11) asm volatile(FOUR(R_OCT) FOUR(R_OCT) FOUR(R_OCT) FOUR(R_OCT) OPS);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[lane] = X ^ Y ^ Z ^ W ^ kh ^ s1 ^ s2 ^ s3 ^ s ^ sk ^ c ^ u ^ m ^ t ^ q.x ^ q.w;
  if (lane == 0) ticks[0] = t1 - t0;
}

template <int V>
static double run(uint32_t* out, uint64_t* ticks) {
  for (int w = 0; w < 20; ++w) k_rounds<V><<<1, 64>>>(out, ticks);
  CHECK(hipDeviceSynchronize());
  uint64_t best = ~0ull;
  for (int r = 0; r < 10; ++r) {
    k_rounds<V><<<1, 64>>>(out, ticks);
    uint64_t h;
    CHECK(hipMemcpy(&h, ticks, 8, hipMemcpyDeviceToHost));
    if (h < best) best = h;
  }
  return (double)best / (kIters * 16.0);
}

int main() {
  uint32_t* out;
  uint64_t* ticks;
  CHECK(hipMalloc(&out, 64 * 4));
  CHECK(hipMalloc(&ticks, 8));
  const char* names[] = {"old11", "new10", "new10v", "valu11", "dpp8", "valu8", "new10b", "new10u", "xad10+nop", "old11+lds", "old11+lds_e", "oct10"};
  const int instrs[] = {11, 10, 10, 11, 8, 8, 10, 10, 11, 11, 11, 10};
  double r[12] = {run<0>(out, ticks), run<1>(out, ticks), run<2>(out, ticks),
                 run<3>(out, ticks), run<4>(out, ticks), run<5>(out, ticks),
                 run<6>(out, ticks), run<7>(out, ticks), run<8>(out, ticks),
                 run<9>(out, ticks), run<10>(out, ticks), run<11>(out, ticks)};
  for (int v = 0; v < 12; ++v)
    printf("{\"variant\": \"%s\", \"instr_per_round\": %d, \"ticks_per_round\": %.2f, \"ticks_per_instr\": %.3f}\n",
           names[v], instrs[v], r[v], r[v] / instrs[v]);
  return 0;
}
