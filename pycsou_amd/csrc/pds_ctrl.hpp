// Device-side loop control of the captured PDS loop (replaces the host `while` of
// GenericIterativeAlgorithm.iterate, pycsou/core/solver.py:65-76, and the diagnostics of
// PrimalDualSplitting.update_diagnostics, pycsou/opt/proxalgs.py:366-394), and the
// in-kernel deterministic reduction of the per-workgroup norm partials.
#pragma once

#include "common.hpp"

namespace pcs {

struct Ctrl {
  int32_t it, stopped, min_iter, max_iter, has_dual, hist_len;
  int32_t pend;  // deferred finalization: the last launch left partials to finalize (fin_slot)
  int32_t pad1;
  double thr;
  double pad2;
};
static_assert(sizeof(Ctrl) == 48, "ctrl layout");

// From the four global sums (||x_old - x||^2, ||x_old||^2, ||z_old - z||^2, ||z_old||^2)
// record the relative improvements of iteration `it`, advance it, and set the sticky stop
// flag exactly when the reference loop would exit.
__device__ __forceinline__ void finalize_from(const double* v, Ctrl* c, double* hist) {
  const int it = c->it;
  const double inf = __builtin_huge_val();
  // ||old - new|| / ||old||, inf if ||old|| == 0 (proxalgs.py:372-383)
  const double rp = (v[1] == 0.0) ? inf : sqrt(v[0]) / sqrt(v[1]);
  const double rd = (v[3] == 0.0) ? inf : sqrt(v[2]) / sqrt(v[3]);
  if (2 * it + 1 < c->hist_len) {
    hist[2 * it] = rp;
    hist[2 * it + 1] = rd;
  }
  const int nx = it + 1;
  c->it = nx;
  // while ((iter <= max_iter) and (stopping_metric() > thr)) or (iter <= min_iter)
  const bool run = (nx <= c->min_iter) || (nx <= c->max_iter && rp > c->thr);
  if (!run || 2 * nx + 1 >= c->hist_len) c->stopped = 1;
}

// ---- in-kernel reduction (hand-off form R1 of cdna_hip_programming.md G16: write-through
// `sc1` payload stores drained by s_waitcnt vmcnt(0) before an agent-scope counter add,
// `sc1` payload loads on the consumer side -- no L2 write-back / invalidate fences, which
// would flush every freshly written x'/z' line of the XCD).
// Workgroups are grouped by blockIdx in groups of kGrp.  Every workgroup publishes its
// 4 partials; the last arriver of a group sums the group's partials in lane order and
// publishes the group sum; the last group sums the group sums in a fixed order and runs
// finalize_from.  Fixed summation order => bitwise-reproducible diagnostics.
// Workspace layout: [ngroups][4] doubles (group sums) | (ngroups + 1) uint32 counters,
// zeroed once before first use; every counter is reset by its last arriver.
// workgroups per group (diagnostics builds override: PCS_RED_GRP).  1024: the one-round grids of the 2-D
// marches (<= 1024 workgroups) reduce in a single level -- one counter round trip and one load round trip at
// the end of the launch instead of two of each: 2048^2 stencil march 28.9-29.5 against 30.0-31.0 us, CPS
// inpainting +5 % (profiles/r5_red_grp_ab.txt); 64 before
#ifndef PCS_RED_GRP
#define PCS_RED_GRP 1024
#endif
constexpr int kGrp = PCS_RED_GRP;

__host__ __device__ inline int64_t red_groups(int64_t nblocks) { return (nblocks + kGrp - 1) / kGrp; }
__host__ __device__ inline int64_t red_ws_bytes(int64_t nblocks) {
  return red_groups(nblocks) * 4 * (int64_t)sizeof(double) + ((red_groups(nblocks) + 1) * 4 + 15) / 16 * 16;
}

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// drain this wave's sc1 stores, then count the arrival
__device__ __forceinline__ unsigned drained_add(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Reduce-only output of the in-kernel reduction (slab mode): the four sums go to `sums`, after
// adding `npre` partials of an earlier launch of the same iteration; no loop control.
struct RedOut {
  double* sums;
  const double* pre;
  int npre;
  const double* fin;  // deferred finalization (single GPU): the previous launch's partials
};

// Entry test of a step kernel against the sticky stop flag (solver.py:65-66): true = skip the
// iterate update.  Plain launches return at once.  A reduce-only launch (slab overlap mode) can
// run while the side stream's loop control writes the flag, so thread 0's reading is broadcast
// and every workgroup still arrives at the reduction counters (with zero partials), which
// then stay consistent for the next run of the plan.
// Single-GPU launches (no sums output) read the stop flag at entry but consume it inside the task, after
// the task's first loads have issued (PCS_DEFER_STOP): the flag's latency overlaps theirs instead of
// preceding them.  The task returns before its first store when the flag is set.
#ifndef PCS_DEFER_STOP
#define PCS_DEFER_STOP 1
#endif
__device__ __forceinline__ bool stop_deferred(const RedOut& ro) { return PCS_DEFER_STOP && ro.sums == nullptr; }
__device__ __forceinline__ int stop_flag_early(const Ctrl* ctrl, const RedOut& ro) {
  return stop_deferred(ro) && ctrl != nullptr ? ctrl->stopped : 0;
}

__device__ __forceinline__ bool stop_requested(const Ctrl* ctrl, const RedOut& ro, int* flag) {
  if (ctrl == nullptr) return false;
  if (ro.sums == nullptr) return ctrl->stopped != 0;
  if (threadIdx.x == 0) flag[0] = __hip_atomic_load(&ctrl->stopped, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return flag[0] != 0;
}

// ---- deferred finalization (single GPU, RedOut::fin non-null; pcs_pds2d_args.fin_partials).
// The step launch of iteration j only stores its workgroups' partials (plain stores, no counters, no
// waiting on the last arriver); an extra workgroup at the head of the NEXT launch (blockIdx 0 of
// kFinBlocks leading slots, so that the tasks keep their XCD mapping) sums them in a fixed order and
// runs finalize_from for iteration j while the tasks of iteration j + 1 run.  When that sets the stop
// flag the reference loop has ended after iteration j: launch j + 1's iterate (written to the other
// parity buffer, which held iterate j - 1) is never selected -- the engines read the iterate of
// parity Ctrl::it -- and its partials are never finalized.  Ctrl::pend says a launch's partials are
// waiting; pcs_pds_finalize_pending finalizes the last launch's at the end of a run.  The partials
// alternate between two arrays with the iterate parity.  Summation order: 256 lanes, lane l adds
// partials l, l + 256, ... in order, then the workgroup tree -- the same in every finalizer.
constexpr int kFinBlocks = 8;
constexpr int kFinLanes = 256;
__device__ __forceinline__ int fin_shift(const RedOut& ro) { return ro.fin != nullptr ? kFinBlocks : 0; }

// `red`: block_sum scratch for the launching kernel's blockDim, `flag`: one int, both LDS
__device__ __forceinline__ void finalize_pending(const double* __restrict__ prev, int64_t nb, Ctrl* c, double* hist,
                                                 bool mark, double* red, int* flag) {
  const int tid = threadIdx.x;
  if (tid == 0) flag[0] = c->pend && !c->stopped;
  __syncthreads();
  if (flag[0]) {  // uniform
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    if (tid < kFinLanes) {
      for (int64_t j = tid; j < nb; j += kFinLanes) {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] += prev[j * 4 + k];
      }
    }
    block_sum<4>(v, red);  // waves past kFinLanes add exact zeros
    if (tid == 0) finalize_from(v, c, hist);
  }
  if (tid == 0) c->pend = mark ? 1 : 0;
}

// Kernel entry of a deferring launch: true for the kFinBlocks leading workgroups (the caller returns);
// workgroup 0 finalizes the previous launch and marks this launch's partials pending.
__device__ __forceinline__ bool fin_slot(const RedOut& ro, int64_t nblocks, Ctrl* ctrl, double* hist, double* red,
                                         int* flag) {
  if (ro.fin == nullptr || blockIdx.x >= kFinBlocks) return false;
  if (blockIdx.x == 0) finalize_pending(ro.fin, nblocks, ctrl, hist, true, red, flag);
  return true;
}

// Called by every thread of every workgroup after thread 0's `part` holds the block sums.
// `flag` is a 2-int LDS scratch.  With ro.sums the last group writes the sums instead of
// running finalize_from.
// ablation (timing only, the loop control never advances; PCS_LIB_PATH builds): 1 = no reduction at all
#ifndef PCS_RED_ABL
#define PCS_RED_ABL 0
#endif
__device__ __forceinline__ void reduce_and_finalize(const double (&part)[4], double* __restrict__ partials,
                                                    int64_t nblocks, void* ws, Ctrl* ctrl, double* hist, int* flag,
                                                    RedOut ro = RedOut{nullptr, nullptr, 0, nullptr}) {
  if (PCS_RED_ABL & 1) return;
  const int tid = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t ngr = red_groups(nblocks);
  double* gsum = reinterpret_cast<double*>(ws);
  unsigned* cnt = reinterpret_cast<unsigned*>(gsum + ngr * 4);
  const int64_t grp = b / kGrp;
  const unsigned members = (unsigned)min<int64_t>(kGrp, nblocks - grp * kGrp);
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) st_sc1(partials + b * 4 + k, part[k]);
    flag[0] = (drained_add(&cnt[grp]) == members - 1);
  }
  __syncthreads();
  if (!flag[0]) return;  // uniform
  __shared__ double red2[4 * 16];
  // ---- last workgroup of its group: thread j sums members j, j + blockDim, ... (fixed order), then the
  // workgroup tree (block_sum)
  {
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = tid; j < (int)members; j += blockDim.x) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] += ld_sc1(partials + (grp * kGrp + j) * 4 + k);
    }
    if (ngr == 1) {  // one group: this workgroup holds the total
      block_sum<4>(v, red2);
      if (tid == 0) __hip_atomic_store(&cnt[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ro.sums != nullptr) {
        double w[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = tid; j < ro.npre; j += blockDim.x) {
#pragma unroll
          for (int k = 0; k < 4; ++k) w[k] += ro.pre[(int64_t)j * 4 + k];
        }
        block_sum<4>(w, red2);
        if (tid == 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) ro.sums[k] = v[k] + w[k];
        }
        return;
      }
      if (tid == 0) finalize_from(v, ctrl, hist);
      return;
    }
    block_sum<4>(v, red2);
    if (tid == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) st_sc1(gsum + grp * 4 + k, v[k]);
      __hip_atomic_store(&cnt[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for next launch
      flag[1] = (drained_add(&cnt[ngr]) == (unsigned)ngr - 1);
    }
  }
  __syncthreads();
  if (!flag[1]) return;  // uniform
  // ---- last group: sum the group sums in a fixed order, then finalize
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t g = tid; g < ngr; g += blockDim.x) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] += ld_sc1(gsum + g * 4 + k);
  }
  block_sum<4>(v, red2);
  if (ro.sums != nullptr) {  // reduce-only: + the earlier launch's partials (fixed order)
    double w[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = tid; j < ro.npre; j += blockDim.x) {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] += ro.pre[(int64_t)j * 4 + k];
    }
    block_sum<4>(w, red2);
    if (tid == 0) {
      __hip_atomic_store(&cnt[ngr], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < 4; ++k) ro.sums[k] = v[k] + w[k];
    }
    return;
  }
  if (tid == 0) {
    __hip_atomic_store(&cnt[ngr], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    finalize_from(v, ctrl, hist);
  }
}

// The end of a step kernel: publish this workgroup's block sums `part` (thread 0's) -- plain partials
// of a deferring launch, the in-kernel reduction with hist / ro.sums, else plain partials.
__device__ __forceinline__ void publish_partials(const double (&part)[4], double* __restrict__ partials,
                                                 int64_t nblocks, void* ws, Ctrl* ctrl, double* hist, int* flag,
                                                 RedOut ro) {
  if (ro.fin == nullptr && (hist != nullptr || ro.sums != nullptr)) {
    reduce_and_finalize(part, partials, nblocks, ws, ctrl, hist, flag, ro);
  } else if (threadIdx.x == 0) {
    const int64_t b = (int64_t)blockIdx.x - fin_shift(ro);
#pragma unroll
    for (int k = 0; k < 4; ++k) partials[b * 4 + k] = part[k];
  }
}

}  // namespace pcs
