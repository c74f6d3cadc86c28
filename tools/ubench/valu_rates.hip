// Issue cost of the instruction kinds the chain and permutation kernels are made of, in SIMD
// cycles per wave64 instruction, at 1, 2 and 8 waves per SIMD.  Every kernel is a loop of 64
// copies of one instruction (or pair); in the plain kernels each copy depends on the one before
// it (one dependency chain per wave), in the *_x2 / *_x4 kernels a wave carries two or four
// independent chains, so that a wave alone can show whether it issues faster than one
// instruction per 4 cycles when its instructions do not wait for each other.
// hipcc --offload-arch=gfx950 -O2 tools/ubench/valu_rates.hip -o valu_rates && ./valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

#define KERNEL(name, body)                                                              \
  __global__ void __launch_bounds__(256) name(int* out, int iters, int seed) {         \
    int a = threadIdx.x + seed, b = a * 3 + 1, c = b ^ 0x55, d = c + 7;                 \
    long long q = ((long long)a << 32) | b;                                             \
    unsigned long long m = 0, m0 = 0x5555aaaa5555aaaaull + seed;                          \
    int sd = seed, sd2 = seed * 5;                                                      \
    float fa = a * 0.5f, fb = 1.0001f, fc = b * 0.25f, fd = c * 0.125f, fe = d * 2.0f;  \
    for (int i = 0; i < iters; i++) {                                                   \
      REP64(body)                                                                       \
    }                                                                                   \
    if (a + b + c + d + sd + sd2 + (int)q + (int)m + (int)m0 + (int)(fa + fb + fc + fd + fe) == 0x7fffffff) out[0] = a; \
  }

KERNEL(k_add, asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_add_x2, asm volatile("v_add_u32 %0, %0, %2\n v_add_u32 %1, %1, %2" : "+v"(a), "+v"(c) : "v"(b));)
KERNEL(k_add_x4, asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                              : "+v"(a), "+v"(c), "+v"(d), "+v"(sd2) : "v"(b));)
KERNEL(k_fma, asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(fa) : "v"(fb));)
KERNEL(k_fma_x2, asm volatile("v_fma_f32 %0, %0, %2, %2\n v_fma_f32 %1, %1, %2, %2" : "+v"(fa), "+v"(fc) : "v"(fb));)
KERNEL(k_fma_x4, asm volatile("v_fma_f32 %0, %0, %4, %4\n v_fma_f32 %1, %1, %4, %4\n v_fma_f32 %2, %2, %4, %4\n v_fma_f32 %3, %3, %4, %4"
                              : "+v"(fa), "+v"(fc), "+v"(fd), "+v"(fe) : "v"(fb));)
KERNEL(k_cndmask_x2, asm volatile("v_cndmask_b32 %0, %0, %2, %3\n v_cndmask_b32 %1, %1, %2, %3" : "+v"(a), "+v"(c) : "v"(b), "s"(m0));)
KERNEL(k_dpp_shl_x2, asm volatile("v_mov_b32_dpp %0, %2 row_shl:1 row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf"
                                  : "+v"(a), "+v"(c) : "v"(b));)
KERNEL(k_cndmask, asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "s"(m0));)
KERNEL(k_and, asm volatile("v_and_b32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_or, asm volatile("v_or_b32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_xor, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_sub, asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_lshl, asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a));)
KERNEL(k_lshr, asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a) : "v"(b));)
KERNEL(k_min, asm volatile("v_min_i32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_max, asm volatile("v_max_u32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_mov, asm volatile("v_mov_b32 %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_addco, asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a) : "v"(b) : "vcc");)
KERNEL(k_and_or, asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
KERNEL(k_lshl_or, asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a) : "v"(b));)
KERNEL(k_add_f32, asm volatile("v_add_f32 %0, %0, %1" : "+v"(fa) : "v"(fb));)
KERNEL(k_mbcnt, asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(a) : "v"(b));)
KERNEL(k_cmp_e64_cnd, asm volatile("v_cmp_lt_i32 %0, %1, %2\n v_cndmask_b32 %1, %1, %2, %0" : "=&s"(m), "+v"(a) : "v"(b));)
KERNEL(k_dpp_shl, asm volatile("v_mov_b32_dpp %0, %1 row_shl:1 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(b));)
KERNEL(k_dpp_bcast, asm volatile("v_mov_b32_dpp %0, %1 row_newbcast:0 row_mask:0xf bank_mask:0x3" : "+v"(a) : "v"(b));)
KERNEL(k_lshr64, asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(q) : "v"(b));)
KERNEL(k_bfe, asm volatile("v_bfe_u32 %0, %0, %1, 8" : "+v"(a) : "v"(b));)
KERNEL(k_perm, asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
KERNEL(k_mul_lo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_mul24, asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(a) : "v"(b));)
KERNEL(k_cmp_vcc, asm volatile("v_cmp_lt_i32 vcc, %0, %1" : : "v"(a), "v"(b) : "vcc");)
KERNEL(k_cmp_sgpr, asm volatile("v_cmp_lt_i32 %0, %1, %2" : "=s"(m) : "v"(a), "v"(b));)
KERNEL(k_cmp_sand, asm volatile("v_cmp_lt_i32 %0, %1, %2\n s_and_b64 %0, %0, exec" : "=s"(m) : "v"(a), "v"(b) : "scc");)
KERNEL(k_cmp_use, asm volatile("v_cmp_lt_i32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");)
KERNEL(k_readlane, asm volatile("v_readlane_b32 %0, %1, 3" : "=s"(sd) : "v"(a));)
KERNEL(k_ffbl, asm volatile("v_ffbl_b32 %0, %0" : "+v"(a));)
KERNEL(k_bperm, asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(a) : "v"(b));)
KERNEL(k_bperm_nowait, asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(c) : "v"(b), "v"(a));)
KERNEL(k_salu, asm volatile("s_add_u32 %0, %0, 1" : "+s"(sd) : : "scc");)
KERNEL(k_lshl_add, asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a) : "v"(b));)
KERNEL(k_add3, asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
KERNEL(k_lshl_add64, asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(q) : "v"(q));)
KERNEL(k_cmp64, asm volatile("v_cmp_lt_u64 vcc, %0, %1" : : "v"(q), "v"(q) : "vcc");)
KERNEL(k_cmp64_addc, asm volatile("v_cmp_lt_u64 vcc, %1, %1\n v_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(a) : "v"(q) : "vcc");)
KERNEL(k_cmp32_addc, asm volatile("v_cmp_lt_u32 vcc, %1, %1\n v_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(a) : "v"(b) : "vcc");)
KERNEL(k_ds_read64, asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(q) : "v"(b));)

int main() {
  int* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  const double ghz = pr.clockRate / 1e6;  // (the nominal clock: a chip that clocks lower under this load shows more cycles)
  const int cus = pr.multiProcessorCount;
  printf("%d CUs at %.3f GHz\n", cus, ghz);
  const int iters = 2000;
  struct { const char* n; void (*k)(int*, int, int); int per; } ks[] = {
      {"v_add_u32", k_add, 1}, {"v_add_u32, 2 chains", k_add_x2, 2}, {"v_add_u32, 4 chains", k_add_x4, 4},
      {"v_fma_f32", k_fma, 1}, {"v_fma_f32, 2 chains", k_fma_x2, 2}, {"v_fma_f32, 4 chains", k_fma_x4, 4},
      {"v_cndmask_b32, 2 chains", k_cndmask_x2, 2}, {"v_mov_dpp row_shl, 2 chains", k_dpp_shl_x2, 2},
      {"v_cndmask_b32 (sgpr mask)", k_cndmask, 1}, {"v_and_b32", k_and, 1}, {"v_or_b32", k_or, 1}, {"v_xor_b32", k_xor, 1},
      {"v_sub_u32", k_sub, 1}, {"v_lshlrev_b32", k_lshl, 1}, {"v_lshrrev_b32", k_lshr, 1}, {"v_min_i32", k_min, 1},
      {"v_max_u32", k_max, 1}, {"v_mov_b32", k_mov, 1}, {"v_add_co_u32", k_addco, 1}, {"v_and_or_b32", k_and_or, 1},
      {"v_lshl_or_b32", k_lshl_or, 1}, {"v_add_f32", k_add_f32, 1}, {"v_mbcnt_lo", k_mbcnt, 1},
      {"v_cmp e64 + v_cndmask (pair)", k_cmp_e64_cnd, 2}, {"v_mov_dpp row_shl", k_dpp_shl, 1},
      {"v_mov_dpp row_newbcast", k_dpp_bcast, 1}, {"v_lshrrev_b64", k_lshr64, 1}, {"v_bfe_u32", k_bfe, 1},
      {"v_perm_b32", k_perm, 1}, {"v_mul_lo_u32", k_mul_lo, 1}, {"v_mul_i32_i24", k_mul24, 1},
      {"v_cmp -> vcc", k_cmp_vcc, 1}, {"v_cmp -> sgpr pair", k_cmp_sgpr, 1}, {"v_cmp + s_and (pair)", k_cmp_sand, 1},
      {"v_cmp + v_cndmask (pair)", k_cmp_use, 1}, {"v_readlane", k_readlane, 1}, {"v_ffbl_b32", k_ffbl, 1},
      {"ds_bpermute + wait", k_bperm, 1}, {"ds_bpermute (no wait)", k_bperm_nowait, 1}, {"s_add_u32", k_salu, 1},
      {"v_lshl_add_u32", k_lshl_add, 1}, {"v_add3_u32", k_add3, 1}, {"v_lshl_add_u64", k_lshl_add64, 1},
      {"v_cmp_lt_u64 -> vcc", k_cmp64, 1}, {"v_cmp_lt_u64 + v_addc (pair)", k_cmp64_addc, 1},
      {"v_cmp_lt_u32 + v_addc (pair)", k_cmp32_addc, 1}, {"ds_read_b64 + wait", k_ds_read64, 1}};
  for (auto& k : ks) {
    for (int wpsimd : {1, 2, 8}) {
      const int blocks = cus * wpsimd;  // 256 threads = 4 waves = one per SIMD of a CU
      k.k<<<blocks, 256>>>(out, 10, 1);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      k.k<<<blocks, 256>>>(out, iters, 1);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double cyc = ms * 1e-3 * ghz * 1e9;            // SIMD cycles of the launch
      const double inst = (double)iters * 64 * wpsimd * k.per;  // instructions per SIMD (`per` in each copy)
      printf("%-28s %d waves/SIMD: %6.2f cycles per wave instruction\n", k.n, wpsimd, cyc / inst);
      fflush(stdout);
    }
  }
  return 0;
}
