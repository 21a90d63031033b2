// calib_fetch.hip -- FETCH_SIZE / WRITE_SIZE calibration for the engine's access width.
// The engine streams fp64 fields with one 8-byte load per lane (global_load_dwordx2) and
// coalesced 8-byte stores.  This kernel reads n doubles and writes n doubles exactly once
// with the same instruction widths, over 512 MiB per array (> the 256 MiB Infinity Cache),
// so rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE can be compared with a known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_calib_copy(const double* __restrict__ a, double* __restrict__ b, long n) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n; q += (long)gridDim.x * blockDim.x)
    b[q] = a[q] * 1.0000001;
}

int main() {
  const long n = 64L << 20;                    // 64 Mi doubles = 512 MiB per array
  double *a, *b;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess) return 1;
  hipMemset(a, 0, n * 8);
  hipMemset(b, 0, n * 8);
  for (int r = 0; r < 3; r++) k_calib_copy<<<8192, 256>>>(a, b, n);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("calib: %ld bytes read, %ld bytes written per launch\n", n * 8, n * 8);
  hipFree(a);
  hipFree(b);
  return 0;
}
