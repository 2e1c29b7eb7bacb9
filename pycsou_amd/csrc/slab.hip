// Native multi-GPU loop of the row-slab 2-D PDS (one process per GPU, RCCL over xGMI).
//
// Replaces, for an image split into row slabs across ranks, the host loop of
//   GenericIterativeAlgorithm.iterate     pycsou/core/solver.py:55-76
// around PrimalDualSplitting.update_iterand / update_diagnostics (pycsou/opt/proxalgs.py:343-394):
// every iteration runs the fused step on this rank's own rows, sums the four norm partials
// across ranks (RCCL all-gather of 4 doubles per rank, added in rank order on every rank, so
// all ranks take the same stop decision) and exchanges the boundary rows of x' and z' with
// the two neighbour ranks (grouped RCCL send/recv).
//
// Overlap mode (row-marching kernels): the boundary bands (the rows the neighbours' halos
// need, and the rows that read our halos) are computed first, then the halo exchange runs on
// a side stream while the interior band is computed on the main stream; the norms all-gather
// and the loop control run on the side stream behind the next iteration's boundary launch.
// That makes iteration i+1 start before iteration i's stop decision is known: it writes only
// the other ping-pong buffers, and iteration i+2 is ordered after that decision (its boundary
// launch waits for the halo exchange that follows it on the side stream), so a stop after
// iteration i leaves iteration i's iterate untouched and every later launch returns at once.
//
// RCCL is bound at run time (dlopen of librccl.so.1: the copy the process already loaded,
// e.g. PyTorch's, or the ROCm one), so the library loads and the single-GPU paths run
// without it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "common.hpp"
#include "pds_ctrl.hpp"

namespace pcs {

struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  bool ok = false;
};

static const Rccl& rccl() {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (h) {
      r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
      r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
      r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
      r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
      r.send = (decltype(r.send))dlsym(h, "ncclSend");
      r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
      r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
      r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
      r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather && r.send && r.recv &&
             r.group_start && r.group_end;
    }
  }
  return r;
}

struct Slab2DPlan {
  pcs_slab2d_desc d;
  ncclComm_t comm;
  hipStream_t side;
  hipEvent_t ev_fork, ev_b, ev_halo, ev_sum, ev_join;
  double* partials;   // [nB + nI] (overlap) or [nfull] partial rows of 4
  double* sums;       // [2][4]
  double* gathered;   // [2][4 world]
  void* ws;           // in-kernel reduction workspace (red_ws_bytes of the reducing launch)
  int64_t nfull, nB, nI;
  bool overlap;
};

static int halo_exchange_on(ncclComm_t comm, int rank, int world, const pcs_halo_set& h, hipStream_t st) {
  const Rccl& R = rccl();
  const int lo = rank - 1, hi = rank + 1;
  const bool has_lo = lo >= 0, has_hi = hi < world;
  if (!has_lo && !has_hi) return PCS_OK;
  if (R.group_start() != ncclSuccess) return PCS_ELAUNCH;
  int bad = 0;
  for (int k = 0; k < h.nbuf; ++k) {
    const size_t nb = (size_t)h.bytes[k];
    if (has_lo) {
      bad |= R.send(h.send_lo[k], nb, ncclUint8, lo, comm, st) != ncclSuccess;
      bad |= R.recv(h.recv_lo[k], nb, ncclUint8, lo, comm, st) != ncclSuccess;
    }
    if (has_hi) {
      bad |= R.send(h.send_hi[k], nb, ncclUint8, hi, comm, st) != ncclSuccess;
      bad |= R.recv(h.recv_hi[k], nb, ncclUint8, hi, comm, st) != ncclSuccess;
    }
  }
  bad |= R.group_end() != ncclSuccess;
  return bad ? PCS_ELAUNCH : PCS_OK;
}

static int halo_exchange(const Slab2DPlan& P, const pcs_halo_set& h, hipStream_t st) {
  return halo_exchange_on(P.comm, P.d.rank, P.d.world, h, st);
}

// argument checks shared by pcs_slab2d_create and pcs_halo_exchange
static bool halo_set_ok(const pcs_halo_set& h, int rank, int world) {
  if (h.nbuf < 0 || h.nbuf > 4) return false;
  for (int k = 0; k < h.nbuf; ++k) {
    if (h.bytes[k] < 0) return false;
    if (rank > 0 && (!h.send_lo[k] || !h.recv_lo[k])) return false;
    if (rank < world - 1 && (!h.send_hi[k] || !h.recv_hi[k])) return false;
  }
  return true;
}

// all-gather of this rank's 4 sums (parity q) + the loop control over the gathered sums
static int sums_and_finalize(const Slab2DPlan& P, int q, hipStream_t st) {
  double* s = P.sums + 4 * q;
  double* g = P.gathered + 4 * (int64_t)P.d.world * q;
  if (P.d.world > 1) {
    if (rccl().all_gather(s, g, 4, ncclFloat64, P.comm, st) != ncclSuccess) return PCS_ELAUNCH;
  } else {
    g = s;
  }
  return pcs_pds_reduce_finalize(g, P.d.world, P.d.ctrl, P.d.hist, st);
}

static int run_serial(Slab2DPlan& P, int64_t n, int p0, hipStream_t st) {
  for (int64_t i = 0; i < n; ++i) {
    const int p = (int)((p0 + i) & 1);
    pcs_pds2d_args a = P.d.step[p];
    a.partials = P.partials;
    a.hist = nullptr;
    a.ws = P.ws;  // the step's last workgroups reduce this rank's partials into sums[p]
    a.sums_out = P.sums + 4 * p;
    a.pre_partials = nullptr;
    a.n_pre = 0;
    int rc = pcs_pds2d_step(&a, st);
    if (rc == PCS_OK) rc = sums_and_finalize(P, p, st);
    if (rc == PCS_OK) rc = halo_exchange(P, P.d.halo[p], st);
    if (rc != PCS_OK) return rc;
  }
  return PCS_OK;
}

static int run_overlap(Slab2DPlan& P, int64_t n, int p0, hipStream_t st) {
  const int64_t R = P.d.step[0].rows, b = P.d.band;
  // the side stream starts behind everything already queued on the caller's stream
  if (hipEventRecord(P.ev_fork, st) != hipSuccess || hipStreamWaitEvent(P.side, P.ev_fork, 0) != hipSuccess)
    return PCS_ELAUNCH;
  for (int64_t i = 0; i < n; ++i) {
    const int p = (int)((p0 + i) & 1);
    pcs_pds2d_args a = P.d.step[p];
    a.hist = nullptr;
    a.ws = nullptr;
    a.sums_out = nullptr;
    // boundary bands: they read the halo rows of iteration i-1
    if (i > 0 && hipStreamWaitEvent(st, P.ev_halo, 0) != hipSuccess) return PCS_ELAUNCH;
    a.partials = P.partials;
    int rc = pcs_pds2d_step_bands(&a, 0, b, R - b, R, st);
    if (rc != PCS_OK) return rc;
    if (hipEventRecord(P.ev_b, st) != hipSuccess) return PCS_ELAUNCH;
    // side: halo exchange of the boundary rows just written, overlapping the interior
    if (hipStreamWaitEvent(P.side, P.ev_b, 0) != hipSuccess) return PCS_ELAUNCH;
    rc = halo_exchange(P, P.d.halo[p], P.side);
    if (rc != PCS_OK) return rc;
    if (hipEventRecord(P.ev_halo, P.side) != hipSuccess) return PCS_ELAUNCH;
    // interior band; its last workgroups reduce its partials + the boundary bands' into sums[p]
    a.partials = P.partials + 4 * P.nB;
    a.ws = P.ws;
    a.sums_out = P.sums + 4 * p;
    a.pre_partials = P.partials;
    a.n_pre = P.nB;
    rc = pcs_pds2d_step_bands(&a, b, R - b, R - b, R - b, st);
    if (rc != PCS_OK) return rc;
    if (hipEventRecord(P.ev_sum, st) != hipSuccess) return PCS_ELAUNCH;
    // side: norms across ranks + stopping rule (the next boundary launch does not wait for it)
    if (hipStreamWaitEvent(P.side, P.ev_sum, 0) != hipSuccess) return PCS_ELAUNCH;
    rc = sums_and_finalize(P, p, P.side);
    if (rc != PCS_OK) return rc;
  }
  // the caller's stream resumes behind the last halo exchange and loop-control update
  if (hipEventRecord(P.ev_join, P.side) != hipSuccess || hipStreamWaitEvent(st, P.ev_join, 0) != hipSuccess)
    return PCS_ELAUNCH;
  return PCS_OK;
}

static void destroy_plan(Slab2DPlan* P) {
  if (!P) return;
  if (P->side) (void)hipStreamDestroy(P->side);
  hipEvent_t* evs[] = {&P->ev_fork, &P->ev_b, &P->ev_halo, &P->ev_sum, &P->ev_join};
  for (hipEvent_t* e : evs)
    if (*e) (void)hipEventDestroy(*e);
  if (P->partials) (void)hipFree(P->partials);
  if (P->sums) (void)hipFree(P->sums);
  if (P->gathered) (void)hipFree(P->gathered);
  if (P->ws) (void)hipFree(P->ws);
  delete P;
}

// ---------------------------------------------------------------- communication-avoiding (deep-halo) loop
// Depth k: x, z (and the static y / Conv^T y) keep halos k iterations deep, so the ranks meet once per k
// iterations instead of once per iteration (the per-iteration all-gather + exchange is ~20-28 us of event
// and RCCL latency, DESIGN.md section 6: the cap of a strongly scaled 4096^2 image).  Iteration j (1..m)
// of a chunk of m <= k iterations computes x', z' on the own rows plus e_j = (m - j) reach redundant halo
// rows each side (clipped at the image), so the own rows after the chunk are exact; the rows each
// iteration adds are the same per-pixel arithmetic as on one GPU (bitwise).  Per iteration two launches of
// the banded step on a "virtual slab" (own rows + e_j): the halo bands (partials discarded) and the own
// band (partials reduced into sums[j]); per chunk one all-gather of the m x 4 sums, the loop control over
// them in iteration order (pcs_pds_reduce_finalize_k) and one exchange of the deep halos.  The buffers
// rotate through nbuf = max(2, k) sets: a natural stop at iteration j of a chunk leaves iterate j intact
// (the chunk's later iterations write the other sets; every launch after the stop flag returns at once).
struct DeepPlan {
  pcs_slab2d_deep_desc d;
  ncclComm_t comm;
  double* part_own = nullptr;  // own-band partials (reduced in-kernel into sums)
  double* part_ext = nullptr;  // halo-band partials (discarded)
  double* sums = nullptr;      // [k][4]
  double* gathered = nullptr;  // [world][k][4]
  void* ws = nullptr;
};

// step b on the virtual slab of own rows + e rows each side (clipped to the image): the row window and
// every halo shrink by s = (lo + hi) / 2 and the bases move by (hi - lo) / 2 rows, so each array's view
// keeps its stored extent (the z component stride rows + 2 halo_z is unchanged)
static pcs_pds2d_args deep_virtual(const DeepPlan& P, int b, int64_t e, int64_t* plo, int64_t* phi) {
  pcs_pds2d_args a = P.d.step[b];
  const int64_t R = a.rows, row0 = a.row0;
  const int64_t up = a.n0 - row0 - R;
  const int64_t lo = e < row0 ? e : row0, hi = e < up ? e : up;
  const int64_t s = (lo + hi) / 2, d = (hi - lo) / 2;
  const int64_t shift = d * a.n1 * (a.dtype == PCS_F64 ? 8 : 4);
  a.row0 = row0 - lo;
  a.rows = R + lo + hi;
  a.halo_x -= (int)s;
  a.halo_z -= (int)s;
  a.halo_y -= (int)s;
  auto sh = [&](const void* q) -> const void* { return q ? (const void*)((const char*)q + shift) : q; };
  a.x = sh(a.x);
  a.xn = (void*)sh(a.xn);
  a.z = sh(a.z);
  a.zn = (void*)sh(a.zn);
  a.y = sh(a.y);
  a.cty = sh(a.cty);
  a.gbuf = sh(a.gbuf);
  a.hist = nullptr;
  a.fin_partials = nullptr;
  a.pre_partials = nullptr;
  a.n_pre = 0;
  *plo = lo;
  *phi = hi;
  return a;
}

// the m iterations of a chunk starting at buffer b0 (launches only)
static int deep_compute(DeepPlan& P, int m, int b0, hipStream_t st) {
  const int B = P.d.nbuf;
  for (int j = 1; j <= m; ++j) {
    const int b = (b0 + j - 1) % B;
    int64_t lo, hi;
    pcs_pds2d_args a = deep_virtual(P, b, (int64_t)(m - j) * P.d.reach, &lo, &hi);
    const int64_t R = P.d.step[b].rows;
    int rc;
    if (lo + hi > 0) {  // the redundant halo rows (their partials are not this rank's)
      a.partials = P.part_ext;
      a.ws = nullptr;
      a.sums_out = nullptr;
      rc = pcs_pds2d_step_bands(&a, 0, lo, lo + R, a.rows, st);
      if (rc != PCS_OK) return rc;
    }
    a.partials = P.part_own;
    a.ws = P.ws;
    a.sums_out = P.sums + 4 * (j - 1);
    rc = lo + hi > 0 ? pcs_pds2d_step_bands(&a, lo, lo + R, lo + R, lo + R, st) : pcs_pds2d_step(&a, st);
    if (rc != PCS_OK) return rc;
  }
  return PCS_OK;
}

static int deep_sync(DeepPlan& P, int m, int b_end, hipStream_t st) {
  const int world = P.d.world;
  if (world > 1) {
    if (rccl().all_gather(P.sums, P.gathered, (size_t)4 * m, ncclFloat64, P.comm, st) != ncclSuccess) return PCS_ELAUNCH;
  } else if (hipMemcpyAsync(P.gathered, P.sums, (size_t)32 * m, hipMemcpyDeviceToDevice, st) != hipSuccess) {
    return PCS_ELAUNCH;
  }
  int rc = pcs_pds_reduce_finalize_k(P.gathered, world, m, P.d.ctrl, P.d.hist, st);
  if (rc == PCS_OK && world > 1) rc = halo_exchange_on(P.comm, P.d.rank, world, P.d.halo[b_end], st);
  return rc;
}

static void destroy_deep(DeepPlan* P) {
  if (!P) return;
  void* bufs[] = {P->part_own, P->part_ext, P->sums, P->gathered, P->ws};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete P;
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int pcs_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int pcs_comm_available(void) { return rccl().ok ? 1 : 0; }

int pcs_comm_unique_id(void* id) {
  if (!id) return PCS_EINVAL;
  if (!rccl().ok) return PCS_EUNSUPPORTED;
  return rccl().get_unique_id((ncclUniqueId*)id) == ncclSuccess ? PCS_OK : PCS_ELAUNCH;
}

int pcs_comm_init(const void* id, int world, int rank, void** comm) {
  if (!id || !comm || world < 1 || rank < 0 || rank >= world) return PCS_EINVAL;
  if (!rccl().ok) return PCS_EUNSUPPORTED;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  if (rccl().comm_init_rank(&c, world, uid, rank) != ncclSuccess) return PCS_ELAUNCH;
  *comm = (void*)c;
  return PCS_OK;
}

int pcs_comm_destroy(void* comm) {
  if (!comm) return PCS_EINVAL;
  if (!rccl().ok) return PCS_EUNSUPPORTED;
  return rccl().comm_destroy((ncclComm_t)comm) == ncclSuccess ? PCS_OK : PCS_ELAUNCH;
}

int pcs_slab2d_create(const pcs_slab2d_desc* d, void* comm, void** plan) {
  if (!d || !plan || d->world < 1 || d->rank < 0 || d->rank >= d->world || !d->ctrl || !d->hist) return PCS_EINVAL;
  if (d->world > 1 && (!comm || !rccl().ok)) return PCS_EINVAL;
  for (int p = 0; p < 2; ++p)
    if (!halo_set_ok(d->halo[p], d->rank, d->world)) return PCS_EINVAL;
  Slab2DPlan* P = new (std::nothrow) Slab2DPlan();
  if (!P) return PCS_ELAUNCH;
  P->d = *d;
  P->comm = (ncclComm_t)comm;
  pcs_pds2d_args a = d->step[0];
  a.hist = nullptr;
  a.ws = nullptr;
  a.sums_out = nullptr;
  a.partials = (double*)d->ctrl;  // non-null placeholder for the argument checks
  P->nfull = pcs_pds2d_nblocks(&a);
  const int64_t R = a.rows, b = d->band;
  P->overlap = false;
  if (d->overlap && b >= 1 && R > 2 * b) {
    P->nB = pcs_pds2d_nblocks_bands(&a, 0, b, R - b, R);
    P->nI = pcs_pds2d_nblocks_bands(&a, b, R - b, R - b, R - b);
    P->overlap = P->nB > 0 && P->nI > 0;
  }
  const int64_t np = P->overlap ? P->nB + P->nI : P->nfull;
  const int64_t wsb = red_ws_bytes(P->overlap ? P->nI : P->nfull);
  bool ok = P->nfull > 0 && hipMalloc(&P->partials, (size_t)np * 4 * sizeof(double)) == hipSuccess &&
            hipMalloc(&P->sums, 8 * sizeof(double)) == hipSuccess &&
            hipMalloc(&P->gathered, (size_t)8 * d->world * sizeof(double)) == hipSuccess &&
            hipMalloc(&P->ws, (size_t)wsb) == hipSuccess && hipMemset(P->ws, 0, (size_t)wsb) == hipSuccess;
  if (ok && P->overlap) {
    ok = hipStreamCreateWithFlags(&P->side, hipStreamNonBlocking) == hipSuccess;
    hipEvent_t* evs[] = {&P->ev_fork, &P->ev_b, &P->ev_halo, &P->ev_sum, &P->ev_join};
    for (hipEvent_t* e : evs) ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
  }
  if (!ok) {
    destroy_plan(P);
    return PCS_ELAUNCH;
  }
  *plan = P;
  return PCS_OK;
}

int pcs_halo_exchange(void* comm, int rank, int world, const pcs_halo_set* h, hipStream_t st) {
  if (!h || world < 1 || rank < 0 || rank >= world || !halo_set_ok(*h, rank, world)) return PCS_EINVAL;
  if (world == 1) return PCS_OK;
  if (!comm || !rccl().ok) return PCS_EINVAL;
  return halo_exchange_on((ncclComm_t)comm, rank, world, *h, st);
}

int pcs_allgather_f64(void* comm, int world, const double* src, double* dst, int64_t count, hipStream_t st) {
  if (!src || !dst || count < 0 || world < 1) return PCS_EINVAL;
  if (!comm) {
    if (world > 1) return PCS_EINVAL;
    return hipMemcpyAsync(dst, src, (size_t)count * sizeof(double), hipMemcpyDeviceToDevice, st) == hipSuccess
               ? PCS_OK
               : PCS_ELAUNCH;
  }
  if (!rccl().ok) return PCS_EINVAL;
  return rccl().all_gather(src, dst, (size_t)count, ncclFloat64, (ncclComm_t)comm, st) == ncclSuccess ? PCS_OK
                                                                                                    : PCS_ELAUNCH;
}

int pcs_slab2d_overlapped(const void* plan) { return plan && ((const Slab2DPlan*)plan)->overlap ? 1 : 0; }

int pcs_slab2d_run(void* plan, int64_t n, int p0, hipStream_t st) {
  if (!plan || n < 0 || (p0 != 0 && p0 != 1)) return PCS_EINVAL;
  Slab2DPlan& P = *(Slab2DPlan*)plan;
  return P.overlap ? run_overlap(P, n, p0, st) : run_serial(P, n, p0, st);
}

int pcs_slab2d_deep_create(const pcs_slab2d_deep_desc* d, void* comm, void** plan) {
  if (!d || !plan || d->world < 1 || d->rank < 0 || d->rank >= d->world || !d->ctrl || !d->hist) return PCS_EINVAL;
  if (d->depth < 1 || d->depth > PCS_DEEP_MAX || d->nbuf < 2 || d->nbuf > PCS_DEEP_MAX || d->nbuf < d->depth)
    return PCS_EINVAL;
  if (d->reach < 1 || d->reach % 2 != 0) return PCS_EINVAL;
  if (d->world > 1 && !d->local && (!comm || !rccl().ok)) return PCS_EINVAL;
  const int64_t R = d->step[0].rows;
  const int64_t emax = (int64_t)(d->depth - 1) * d->reach;
  for (int b = 0; b < d->nbuf; ++b) {
    const pcs_pds2d_args& a = d->step[b];
    if (!halo_set_ok(d->halo[b], d->rank, d->world) || a.rows != R || a.hist || a.fin_partials) return PCS_EINVAL;
    // the stored halos cover the first iteration's extension plus one iteration's reach; a neighbour's
    // slab is at least that thick (the exchange sends own rows), so clipping leaves lo, hi in {0, e}
    if (a.halo_x < emax + 1 || a.halo_z < emax + 1 || a.halo_y < emax + 1 || R < a.halo_x || R < a.halo_z)
      return PCS_EINVAL;
  }
  DeepPlan* P = new (std::nothrow) DeepPlan();
  if (!P) return PCS_ELAUNCH;
  P->d = *d;
  P->comm = (ncclComm_t)comm;
  int64_t nown = 0, next = 0;
  for (int b = 0; b < d->nbuf && b < 2; ++b) {
    for (int j = 0; j < d->depth; ++j) {
      int64_t lo, hi;
      pcs_pds2d_args a = deep_virtual(*P, b, (int64_t)j * d->reach, &lo, &hi);
      a.partials = (double*)d->ctrl;  // non-null placeholder for the argument checks
      const int64_t no = lo + hi > 0 ? pcs_pds2d_nblocks_bands(&a, lo, lo + R, lo + R, lo + R) : pcs_pds2d_nblocks(&a);
      const int64_t ne = lo + hi > 0 ? pcs_pds2d_nblocks_bands(&a, 0, lo, lo + R, a.rows) : 0;
      if (no < 1 || ne < 0) {
        destroy_deep(P);
        return PCS_EUNSUPPORTED;  // the banded (row-marching) step does not take these arguments
      }
      nown = no > nown ? no : nown;
      next = ne > next ? ne : next;
    }
  }
  const int64_t wsb = red_ws_bytes(nown);
  bool ok = hipMalloc(&P->part_own, (size_t)nown * 32) == hipSuccess &&
            hipMalloc(&P->part_ext, (size_t)(next > 0 ? next : 1) * 32) == hipSuccess &&
            hipMalloc(&P->sums, (size_t)32 * d->depth) == hipSuccess &&
            hipMalloc(&P->gathered, (size_t)32 * d->depth * d->world) == hipSuccess &&
            hipMalloc(&P->ws, (size_t)wsb) == hipSuccess && hipMemset(P->ws, 0, (size_t)wsb) == hipSuccess;
  if (!ok) {
    destroy_deep(P);
    return PCS_ELAUNCH;
  }
  *plan = P;
  return PCS_OK;
}

int pcs_slab2d_deep_run(void* plan, int64_t n, int b0, hipStream_t st) {
  if (!plan || n < 0) return PCS_EINVAL;
  DeepPlan& P = *(DeepPlan*)plan;
  if (b0 < 0 || b0 >= P.d.nbuf || (P.d.local && P.d.world > 1)) return PCS_EINVAL;
  while (n > 0) {
    const int m = (int)(n < P.d.depth ? n : P.d.depth);
    int rc = deep_compute(P, m, b0, st);
    b0 = (b0 + m) % P.d.nbuf;
    if (rc == PCS_OK) rc = deep_sync(P, m, b0, st);
    if (rc != PCS_OK) return rc;
    n -= m;
  }
  return PCS_OK;
}

int pcs_slab2d_deep_run_local(void* const* plans, int nplans, int64_t n, int b0, hipStream_t st) {
  if (!plans || nplans < 1 || nplans > 64 || n < 0) return PCS_EINVAL;
  DeepPlan* by_rank[64] = {nullptr};
  const DeepPlan& P0 = *(const DeepPlan*)plans[0];
  for (int i = 0; i < nplans; ++i) {
    DeepPlan* P = (DeepPlan*)plans[i];
    if (!P || P->d.world != nplans || P->d.depth != P0.d.depth || P->d.nbuf != P0.d.nbuf || by_rank[P->d.rank])
      return PCS_EINVAL;
    by_rank[P->d.rank] = P;
  }
  if (b0 < 0 || b0 >= P0.d.nbuf) return PCS_EINVAL;
  auto cp = [&](void* dst, const void* src, int64_t bytes) {
    return hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, st) == hipSuccess;
  };
  while (n > 0) {
    const int m = (int)(n < P0.d.depth ? n : P0.d.depth);
    for (int r = 0; r < nplans; ++r) {
      const int rc = deep_compute(*by_rank[r], m, b0, st);
      if (rc != PCS_OK) return rc;
    }
    b0 = (b0 + m) % P0.d.nbuf;
    // the transport of deep_sync, device to device: all-gather of the sums, then the deep halos
    for (int r = 0; r < nplans; ++r)
      for (int q = 0; q < nplans; ++q)
        if (!cp(by_rank[r]->gathered + (int64_t)q * 4 * m, by_rank[q]->sums, 32 * m)) return PCS_ELAUNCH;
    for (int r = 0; r < nplans; ++r) {
      const int rc = pcs_pds_reduce_finalize_k(by_rank[r]->gathered, nplans, m, by_rank[r]->d.ctrl,
                                               by_rank[r]->d.hist, st);
      if (rc != PCS_OK) return rc;
    }
    for (int r = 0; r + 1 < nplans; ++r) {  // r's last rows -> r + 1's lower halo, r + 1's first rows -> r's upper
      const pcs_halo_set& a = by_rank[r]->d.halo[b0];
      const pcs_halo_set& b = by_rank[r + 1]->d.halo[b0];
      for (int k = 0; k < a.nbuf; ++k)
        if (!cp(b.recv_lo[k], a.send_hi[k], a.bytes[k]) || !cp(a.recv_hi[k], b.send_lo[k], b.bytes[k]))
          return PCS_ELAUNCH;
    }
    n -= m;
  }
  return PCS_OK;
}

int pcs_slab2d_deep_destroy(void* plan) {
  if (!plan) return PCS_EINVAL;
  destroy_deep((DeepPlan*)plan);
  return PCS_OK;
}

int pcs_slab2d_destroy(void* plan) {
  if (!plan) return PCS_EINVAL;
  destroy_plan((Slab2DPlan*)plan);
  return PCS_OK;
}

}  // extern "C"
