// What the HBM delivers to simple streaming kernels on this GPU, to set beside the bandwidth-
// bound codec kernels: a pure read (16 B per lane, coalesced), a read of one 4-byte word of
// every 32-byte record (the histogram pass), a copy, a read + half-size write (the
// scatter's 32 B in, 17 B out), a pure write and a read + double-size write.  Buffers are far larger than the caches.
// hipcc --offload-arch=gfx950 -O3 tools/ubench/hbm_rates.hip -o hbm_rates && ./hbm_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void __launch_bounds__(256) k_read16(const int4* __restrict__ in, long n, int* out) {
  int acc = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int4 v = in[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x7ffffff1) out[0] = acc;
}
__global__ void __launch_bounds__(256) k_read4of32(const int* __restrict__ in, long nrec, int* out) {
  int acc = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nrec; i += (long)gridDim.x * 256) acc += in[i * 8 + 7];
  if (acc == 0x7ffffff1) out[0] = acc;
}
__global__ void __launch_bounds__(256) k_copy16(const int4* __restrict__ in, int4* __restrict__ o, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) o[i] = in[i];
}
__global__ void __launch_bounds__(256) k_read32_write16(const int4* __restrict__ in, int4* __restrict__ o, long nrec) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nrec; i += (long)gridDim.x * 256) {
    const int4 a = in[2 * i], b = in[2 * i + 1];
    o[i] = make_int4(a.x + b.x, a.y + b.y, a.z ^ b.z, a.w ^ b.w);
  }
}

__global__ void __launch_bounds__(256) k_write16(int4* __restrict__ o, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) o[i] = make_int4((int)i, 1, 2, 3);
}
__global__ void __launch_bounds__(256) k_read16_write32(const int4* __restrict__ in, int4* __restrict__ o, long nrec) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < nrec; i += (long)gridDim.x * 256) {
    const int4 a = in[i];
    o[2 * i] = a;
    o[2 * i + 1] = make_int4(a.w, a.z, a.y, a.x);
  }
}

int main() {
  const long bytes = 6l << 30;
  int4 *a, *b;
  int* out;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(a, 1, bytes));
  CHECK(hipMemset(b, 2, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const long n16 = bytes / 16, nrec = bytes / 32;
  for (int grid : {2048, 8192, 32768}) {
    for (int k = 0; k < 6; k++) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; rep++) {
        CHECK(hipEventRecord(e0));
        if (k == 0) k_read16<<<grid, 256>>>(a, n16, out);
        if (k == 1) k_read4of32<<<grid, 256>>>((const int*)a, nrec, out);
        if (k == 2) k_copy16<<<grid, 256>>>(a, b, n16);
        if (k == 3) k_read32_write16<<<grid, 256>>>(a, b, nrec);
        if (k == 4) k_write16<<<grid, 256>>>(b, n16);
        if (k == 5) k_read16_write32<<<grid, 256>>>(a, b, nrec);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      const double moved = k == 0 ? bytes : k == 1 ? bytes : k == 2 ? 2.0 * bytes : k == 4 ? bytes : 1.5 * bytes;
      const char* names[] = {"read 16 B/lane", "read 4 of every 32 B (bytes of the records)", "copy 16 B/lane (read + write)",
                             "read 32 B + write 16 B per record", "write 16 B/lane",
                             "read 16 B + write 32 B per record (the decoder's last pass)"};
      printf("grid %6d  %-44s %7.3f ms  %6.2f TB/s\n", grid, names[k], best, moved / best / 1e9);
    }
  }
  return 0;
}
