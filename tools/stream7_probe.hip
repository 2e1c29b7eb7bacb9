// Practical HBM roofline for the fused PDS step's traffic mix (diagnostics, GPU box):
// read x, y, z0, z1 and write x', z0', z1' (7 fp32 words per pixel, 4096^2 pixels = 470 MB),
// elementwise, 16-B per lane, every CU busy.  Also a plain copy (1 read + 1 write) for scale.
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream7_probe.bin tools/stream7_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k7(const f4* __restrict__ x, const f4* __restrict__ y, const f4* __restrict__ z0,
                                          const f4* __restrict__ z1, f4* __restrict__ xn, f4* __restrict__ zn0,
                                          f4* __restrict__ zn1, long n4, float a) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const f4 xv = x[i], yv = y[i], z0v = z0[i], z1v = z1[i];
    xn[i] = xv + a * yv;
    zn0[i] = z0v + a * xv;
    zn1[i] = z1v + a * yv;
  }
}

__global__ __launch_bounds__(256) void kcopy(const f4* __restrict__ x, f4* __restrict__ xn, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) xn[i] = x[i];
}

int main() {
  const long n = 4096L * 4096L, n4 = n / 4;
  std::vector<f4*> b(7);
  for (auto& p : b) {
    hipMalloc(&p, n * 4);
    hipMemset(p, 0, n * 4);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int per_cu : {2, 4, 8, 16, 32}) {
    const int grid = cus * per_cu;
    for (int w = 0; w < 20; ++w) k7<<<grid, 256>>>(b[0], b[1], b[2], b[3], b[4], b[5], b[6], n4, 0.5f);
    std::vector<float> t;
    for (int r = 0; r < 50; ++r) {
      hipEventRecord(e0);
      k7<<<grid, 256>>>(b[0], b[1], b[2], b[3], b[4], b[5], b[6], n4, 0.5f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf("stream7 grid %5d (%2d/CU): median %.1f us = %.2f TB/s (7 words/px)\n", grid, per_cu, med * 1e3,
           7.0 * n * 4 / (med * 1e-3) / 1e12);
    t.clear();
    for (int r = 0; r < 50; ++r) {
      hipEventRecord(e0);
      kcopy<<<grid, 256>>>(b[0], b[4], n4);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double mc = t[t.size() / 2];
    printf("copy    grid %5d (%2d/CU): median %.1f us = %.2f TB/s\n", grid, per_cu, mc * 1e3,
           2.0 * n * 4 / (mc * 1e-3) / 1e12);
  }
  return 0;
}
