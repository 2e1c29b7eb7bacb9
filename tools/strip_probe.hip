// Access-pattern probe (round 6): does the row-segment width a workgroup streams decide the HBM rate?
// Four 4096^2 fp32 inputs and three outputs (the C3 step's x, b, z0, z1 in / x', z0', z1' out) are streamed
// by workgroups that march down strips of W columns, 16 rows per step (as k_pds2d_nmarch does with W = 64),
// against a flat grid-stride stream of the same bytes.  No LDS, no arithmetic beyond a sum: memory alone.
//   hipcc --offload-arch=gfx950 -O3 -o tools/strip_probe tools/strip_probe.hip && tools/strip_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int N = 4096;

struct Arr {
  const float4* in[4];
  float4* out[3];
};

// task = (segment, strip); rows [seg * L, seg * L + L) of columns [strip * W, strip * W + W)
template <int W>
__global__ __launch_bounds__(256) void k_strips(Arr a, int nstrips, int L) {
  constexpr int G = W / 4;              // float4 groups per row
  constexpr int RPS = 256 / G;          // rows one pass of the workgroup covers (W <= 1024)
  const int task = blockIdx.x, seg = task / nstrips, strip = task - seg * nstrips;
  const int g = threadIdx.x % G, r0 = threadIdx.x / G;
  const int64_t col4 = (int64_t)strip * G + g;
  const int end = min(seg * L + L, N);
  for (int r = seg * L + r0; r < end; r += RPS) {
    const int64_t o = (int64_t)r * (N / 4) + col4;
    const float4 v0 = a.in[0][o], v1 = a.in[1][o], v2 = a.in[2][o], v3 = a.in[3][o];
    a.out[0][o] = make_float4(v0.x + v1.x, v0.y + v1.y, v0.z + v1.z, v0.w + v1.w);
    a.out[1][o] = make_float4(v2.x + v3.x, v2.y + v3.y, v2.z + v3.z, v2.w + v3.w);
    a.out[2][o] = make_float4(v0.x + v3.x, v0.y + v3.y, v0.z + v3.z, v0.w + v3.w);
  }
}

__global__ __launch_bounds__(256) void k_flat(Arr a, int64_t n4) {
  for (int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x; o < n4; o += (int64_t)gridDim.x * 256) {
    const float4 v0 = a.in[0][o], v1 = a.in[1][o], v2 = a.in[2][o], v3 = a.in[3][o];
    a.out[0][o] = make_float4(v0.x + v1.x, v0.y + v1.y, v0.z + v1.z, v0.w + v1.w);
    a.out[1][o] = make_float4(v2.x + v3.x, v2.y + v3.y, v2.z + v3.z, v2.w + v3.w);
    a.out[2][o] = make_float4(v0.x + v3.x, v0.y + v3.y, v0.z + v3.z, v0.w + v3.w);
  }
}

template <typename F>
static float time_ms(F launch, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms / reps;
}

template <int W>
static void run_strips(const Arr& a, int ntasks_target, int reps) {
  const int nstrips = N / W;
  int nseg = ntasks_target / nstrips;
  nseg = nseg < 1 ? 1 : nseg;
  const int L = (N + nseg - 1) / nseg;
  const double bytes = 7.0 * N * (double)N * 4;
  const float ms = time_ms([&] { k_strips<W><<<nstrips * nseg, 256>>>(a, nstrips, L); }, reps);
  printf("{\"pattern\": \"strips\", \"W\": %d, \"row_bytes\": %d, \"tasks\": %d, \"seg_rows\": %d, \"us\": %.2f, \"TBps\": %.3f}\n",
         W, W * 4, nstrips * nseg, L, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
}

int main() {
  Arr a;
  const size_t bytes = (size_t)N * N * 4;
  for (int k = 0; k < 4; ++k) {
    void* p;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    a.in[k] = (const float4*)p;
  }
  for (int k = 0; k < 3; ++k) {
    void* p;
    CK(hipMalloc(&p, bytes));
    a.out[k] = (float4*)p;
  }
  const int reps = 50;
  const double tot = 7.0 * bytes;
  for (int pass = 0; pass < 2; ++pass) {
    const float ms = time_ms([&] { k_flat<<<4096, 256>>>(a, (int64_t)N * N / 4); }, reps);
    printf("{\"pattern\": \"flat\", \"us\": %.2f, \"TBps\": %.3f}\n", ms * 1e3, tot / (ms * 1e-3) / 1e12);
    for (int t : {768, 1536, 4096}) {
      printf("# tasks target %d\n", t);
      run_strips<64>(a, t, reps);
      run_strips<128>(a, t, reps);
      run_strips<256>(a, t, reps);
      run_strips<512>(a, t, reps);
      run_strips<1024>(a, t, reps);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
