// Round 5: accuracy of the fp64 fast_rsqrt (pds_tile.hpp: v_rsq_f64 + two Newton steps) against 1 / sqrt in
// long double on the host, over 2^20 values spread across [1e-300, 1e300] plus 0 and +inf.  Prints the largest
// relative error (in ulps of the correctly rounded result).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../pycsou_amd/csrc/common.hpp"
#include "../pycsou_amd/csrc/pds_tile.hpp"
__global__ void k(const double* v, double* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = pcs::fast_rsqrt(v[i]);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> v(n), o(n);
  srand(1);
  for (int i = 0; i < n; ++i) v[i] = std::pow(10.0, -300.0 + 600.0 * (rand() / (double)RAND_MAX)) * (1.0 + rand() / (double)RAND_MAX);
  v[0] = 0.0;
  v[1] = HUGE_VAL;
  v[2] = 1.0;
  v[3] = 4.0;
  double *dv, *dout;
  if (hipMalloc(&dv, n * 8) != hipSuccess || hipMalloc(&dout, n * 8) != hipSuccess) return 2;
  if (hipMemcpy(dv, v.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess) return 3;
  k<<<n / 256, 256>>>(dv, dout, n);
  if (hipMemcpy(o.data(), dout, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  double worst = 0.0;
  for (int i = 2; i < n; ++i) {
    const long double r = 1.0L / sqrtl((long double)v[i]);
    const double rd = (double)r;
    const double ulp = std::nextafter(rd, HUGE_VAL) - rd;
    const double e = std::fabs((double)((long double)o[i] - r)) / ulp;
    if (e > worst) worst = e;
  }
  printf("fast_rsqrt(0) = %g, fast_rsqrt(inf) = %g, rsqrt(4) = %.17g, max error %.3f ulp over %d values\n", o[0], o[1],
         o[3], worst, n - 2);
  return (std::isinf(o[0]) && o[1] == 0.0 && worst <= 2.0) ? 0 : 1;
}
