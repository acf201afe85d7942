// mvba_solve.cpp — GPU-resident Levenberg-Marquardt driver (mvba_solve).
//
// Replaces ceres::Solve with linear_solver_type = ITERATIVE_SCHUR and the
// default JACOBI preconditioner (rig_calibrator.cc:1910-1919) for problems of
// BracketedCamError blocks. Control flow follows Ceres 1.14 [ext, not vendored]:
//   trust_region_minimizer.cc     Minimize / IterationZero / ComputeTrustRegionStep /
//                                 ParameterToleranceReached / FunctionToleranceReached /
//                                 HandleSuccessfulStep / HandleInvalidStep, Jacobi
//                                 column scaling fixed at iteration 0;
//   levenberg_marquardt_strategy.cc  diagonal clamp, radius update
//                                 radius /= max(1/3, 1-(2rho-1)^3), reject: /= 2,4,8...;
//   iterative_schur_complement_solver.cc + implicit_schur_complement.cc
//                                 CG on S = F'F + D_f^2 - F'E (E'E + D_e^2)^-1 E'F with
//                                 the block-diagonal (F'F + D_f^2)^-1 preconditioner;
//   conjugate_gradients_solver.cc  q-criterion termination (eta), residual reset every 10;
//   line_search.cc (ArmijoLineSearch)  projected line search when bounds are active.
// All vectors live in HBM; the host only sees scalars (dot products, costs).
#include <algorithm>
#include <chrono>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>

#include "mvba_internal.h"

extern "C" {
int mvba_solver_dir_stride(void);
int mvba_solver_vec_replicas(void);
int64_t mvba_pass_a_blocks(int64_t npts);
hipError_t mvba_launch_frame_dir(const void* fl, int32_t nframes, const FrameDesc* fd, const double* frec,
                                 const double* x, double* dir, const int32_t* gate, const mvba::LazyDir* lz,
                                 hipStream_t s);
hipError_t mvba_launch_pass_a(int model, int deg, const int64_t* pt_begin, int64_t npts, const int32_t* po_frame,
                              const double2* po_meas, const FrameDesc* fd, const double* frec,
                              const double* params, const double4* pts, const double* dir, const double* tinit,
                              const double* V, const double* dp, double* zbuf, double* wout, int32_t wstride,
                              double* sq_partial, unsigned* counter, double* sq_out, int32_t flags, double cauchy_c,
                              mvba::PointExtra dc, const double* xcam, double* du, const int32_t* gate,
                              const double* prec, hipStream_t s);
hipError_t mvba_launch_pass_a_frame(int model, int deg, const int4* chunks, int32_t nchunks,
                                    const mvba::Segment* segs, const double4* pts, const int32_t* obs_pid,
                                    const double2* obs_meas, const int32_t* slot_po, mvba::DirPair dir,
                                    double4* cbuf, int32_t flags, double cauchy_c, const int32_t* gate,
                                    const double* prec, const double4* obsX, hipStream_t s);
hipError_t mvba_launch_pass_sq(int model, int deg, const int4* chunks, int32_t nchunks, const int32_t* obs_pid,
                               mvba::DirPair dir, const double* wbuf, int32_t wstride, const double* prec,
                               const double4* obsX, double* partial, unsigned* counter, double* sq_out,
                               hipStream_t s);
hipError_t mvba_launch_point_w(int64_t npts, const int64_t* pt_begin, const int32_t* po_slot, const double4* cbuf,
                               const double* tinit, const double* V, const double* dp, const double4* pts,
                               double* wout, int32_t wstride, const int32_t* gate, const int64_t* dbegin,
                               const double4* dcbuf, const mvba::FusedStep* fs, hipStream_t s);
hipError_t mvba_launch_upd_pass_a(int model, int deg, int64_t n, const mvba::CgEntry* ent, const double* minv,
                                  const double* p, const double* q, const double* b, double* x, const double* r_in,
                                  double* r_out, double* z, double* partial, unsigned* counters, double* out,
                                  mvba::CgCtl* ctl, const double* pq_in, const int4* chunks, int32_t nchunks,
                                  const void* fl, const mvba::FrameDesc* fd, const double* frec, const double* dp,
                                  double* dz_out, const int32_t* slot_po, double4* cbuf, double* cbuf2,
                                  const double* prec, const double4* obsX, hipStream_t s);
hipError_t mvba_launch_point_w_seg(int32_t ntiles, const int4* tiles, const int32_t* wlane_pid,
                                   const int32_t* wlane_idx, const int64_t* pt_begin, const int32_t* po_idx,
                                   const double4* cbuf, const double* tinit, const double* V, const double* dp,
                                   const double4* pts, double* wout, int32_t wstride, const int32_t* gate,
                                   hipStream_t s);
hipError_t mvba_launch_depth_pa(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                const int32_t* dpid, const double4* dmeas, const double* frec, const double* params,
                                const double4* pts, const double* dir, const double* xcam, double* du,
                                const int32_t* dslot_po, double4* dcbuf, int32_t flags, double cauchy_c,
                                const int32_t* gate, hipStream_t s);
hipError_t mvba_launch_frame_proj(int32_t nframes, const mvba::FrameDesc* fd, const double* frec,
                                  const double* params, double* prec, hipStream_t s);
hipError_t mvba_launch_depth_sb(const mvba::Segment* segs, int32_t nseg, const mvba::DepthDesc* dd,
                                const int32_t* dpid, const double4* dmeas, const double* frec, const double* params, const double4* pts,
                                const void* fl, const double* du, double* yrep, int64_t ng, int32_t flags,
                                double cauchy_c, const int32_t* gate, mvba::Slab sl, const double4* wbuf,
                                hipStream_t s);
hipError_t mvba_launch_pass_b(int model, int deg, const int4* chunks, int32_t nchunks, int32_t chunk_base,
                              const Segment* segs, const FrameDesc* fd, const void* fl, const double* frec,
                              const double* params, const double4* pts, const int32_t* obs_pid,
                              const double2* obs_meas, const double* dir, const double4* wbuf, double* yrep,
                              int64_t ng, int32_t flags, double cauchy_c, const int32_t* gate, mvba::Slab sl,
                              const double4* obsX, hipStream_t s);
hipError_t mvba_launch_slab_reduce_vec(mvba::SlabTiers t, int64_t grid, const int64_t* begin, const int64_t* pos,
                                       const double* val, const double* diag, const double* x, double* y,
                                       double* partial, unsigned* counter, double* dot_out, const int32_t* gate,
                                       mvba::CgCtl* ctl, const mvba::LazyDir* lz, int32_t local_dot, hipStream_t s);
hipError_t mvba_launch_rep_reduce_vec(double* yrep, int64_t ng, const double* diag, const double* x, double* y,
                                      double* partial, unsigned* counter, double* dot_out, const int32_t* gate,
                                      mvba::CgCtl* ctl, const mvba::LazyDir* lz, int32_t local_dot,
                                      double* dot_zero, hipStream_t s);
hipError_t mvba_launch_add_diag(int64_t n, const double* diag, const double* x, double* y, double* partial,
                                unsigned* counter, double* dot_out, const int32_t* gate, mvba::CgCtl* ctl,
                                const mvba::LazyDir* lz, hipStream_t s);
hipError_t mvba_launch_cg_update(int64_t n, const mvba::CgEntry* ent, const double* minv, int32_t mode, double alpha,
                                 const double* p,
                                 const double* q, const double* b, double* x, const double* r_in, double* r_out,
                                 double* z, double* partial, unsigned* counters, double* out, mvba::CgCtl* ctl,
                                 int32_t iter, const mvba::FrameDirZ* fz, const double* pq_in, mvba::CgMirror* mir,
                                 hipStream_t s);
hipError_t mvba_launch_axpby(int64_t n, double a, const double* x, double b, const double* y, double* out,
                             hipStream_t s);
hipError_t mvba_launch_dot(int64_t n, const double* x, const double* y, double* partial, unsigned* counter, double* out,
                           hipStream_t s);
hipError_t mvba_launch_sum(int64_t n, double* partial, double* out, hipStream_t s);
hipError_t mvba_launch_block_prec(int32_t nblocks, int32_t max_bsize, const int64_t* goff, const int64_t* hoff,
                                  const int32_t* bsize, const double* hess, const double* d, double* minv,
                                  hipStream_t s);
hipError_t mvba_launch_extract_diag(int32_t nblocks, const int64_t* goff, const int64_t* hoff, const int32_t* bsize,
                                    const double* hess, int64_t npts, const double* V, int64_t ng, double* c,
                                    hipStream_t s);
hipError_t mvba_launch_jacobi_scale(int64_t n, const double* c, double* sc, hipStream_t s);
hipError_t mvba_launch_lm_diag(int64_t n, const double* c, const double* sc, double inv_radius,
                               const double* inv_radius_dev, double dmin, double dmax, double* d, hipStream_t s);
hipError_t mvba_launch_gather(int64_t ncam, const int64_t* cam_poff, int64_t npts, const int64_t* pt_off,
                              const uint8_t* pt_free, const double* params, double* out, hipStream_t s);
hipError_t mvba_launch_scatter(int64_t ncam, const int64_t* cam_poff, int64_t npts, const int64_t* pt_off,
                               const uint8_t* pt_free, const double* in, double* params, hipStream_t s);
hipError_t mvba_launch_plus(int64_t n, const double* x, const double* delta, const double* lower,
                            const double* upper, double* out, hipStream_t s);
hipError_t mvba_launch_proj_grad_max(int64_t n, const double* x, const double* g, const double* lower,
                                     const double* upper, double* partial, double* out, hipStream_t s);
hipError_t mvba_launch_cost(int model, int deg, const Segment* segs, int32_t nseg, const FrameDesc* fd,
                            const double* frec, const double* params, const double4* pts, const int32_t* obs_pid,
                            const double2* obs_meas, int32_t flags, double cauchy_c, double* partial, hipStream_t s,
                            int64_t* nblocks_out);
}

// Device + pinned host state of one handle's solver (allocated by the first mvba_solve).
struct SolverState {
  int64_t ng = 0, nh = 0, np = 0, nc = 0;  // camera grad/hess sizes, points, compact size ng + 3 np
  int32_t nblocks = 0;
  double* lin = nullptr;      // [ng | nh | 1]: camera gradient, block Hessians, cost (one all-reduce)
  double* phess = nullptr;    // [6 np] point Hessians V_p
  double* G = nullptr;        // [nc] compact gradient
  double* cdiag = nullptr;    // [nc] diag(J^T J)
  double* sc = nullptr;       // [nc] Jacobi scaling (iteration 0)
  double* dmp = nullptr;      // [nc] LM damping (unscaled)
  double* fac = nullptr;      // [nh] explicit inverses of the preconditioner blocks
  double* x = nullptr;        // [nc] current point (compact)
  double* xn = nullptr;       // [nc] candidate point
  double* delta = nullptr;    // [nc] step (camera part = CG solution)
  double* scr = nullptr;      // [nc] scratch
  double* lo = nullptr;       // [nc] bounds (compact) or null
  double* hi = nullptr;
  double *b = nullptr, *r = nullptr, *r2 = nullptr, *z = nullptr, *p = nullptr, *p2 = nullptr, *q = nullptr,
         *tmp = nullptr;  // [ng]; p, p2: the CG direction, double-buffered
  double* yrep = nullptr;     // [replicas * ng], kept zero between products
  double* dir = nullptr;      // [nframes * dir stride]
  double* dirz = nullptr;     // [nframes * dir stride] W z, by the CG update's frame blocks
  double* dirp[2] = {nullptr, nullptr};  // W p_old / W p_new, alternating CG products
  double* zbuf = nullptr;     // [8 N] point-order z_o | J_pt rows
  double* wbuf = nullptr;     // [4 np] w_p of the last pass A (double4 per point)
  double* cbuf = nullptr;     // [4 slots] frame-order pass A: J_pt^T z per slot
  double* cbuf2 = nullptr;    // [2 slots] the fused CG step's second product (c_p.y, c_p.z)
  double* obsX = nullptr;     // [4 slots] landmark of each slot (fixed during a linear solve)
  double* du = nullptr;       // [3 depth slots] u_d (point-order pass A) or z_d (k_depth_pa) -> k_depth_sb
  double* dcbuf = nullptr;    // [4 depth blocks] P z_d at the point-order position (k_depth_pa -> k_point_w)
  double* partial = nullptr;  // [npartial]
  double* scal = nullptr;     // [32] device scalars; [24..25]: the CG's p.q accumulators (kPqSlot)
  unsigned* cnt = nullptr;    // [8] grid-reduction counters (kept zero between kernels)
  double* hscal = nullptr;    // [32] pinned host mirror
  mvba::CgCtl* ctl = nullptr; // device CG control (single-rank solves)
  mvba::CgCtl* ctl0 = nullptr; // the solve's initial control block (options only; copied to ctl per linear solve)
  double* prec = nullptr;     // [nframes * kProjDoubles] projection records
  mvba::CgCtl* hctl = nullptr; // pinned host mirror
  // host-coherent mapped CgMirror the batches' last update launches write
  // (hmir: host address, dmir: its device address)
  mvba::CgMirror* hmir = nullptr;
  mvba::CgMirror* dmir = nullptr;
  int64_t npartial = 0;
  int32_t* bsize = nullptr;
  mvba::CgEntry* ent = nullptr;  // per camera entry: block start, size, inverse row
  int32_t max_bsize = 0;
  int64_t *goff = nullptr, *hoff = nullptr, *cam_poff = nullptr;
  DetPlan b_det;              // deterministic pass B (slab rows per chunk / depth segment)
  // Captured CG iteration runs (hipGraph): iterations at offsets [o, o + L) of
  // a 10-iteration period (Ceres' residual reset), replayed by one
  // hipGraphLaunch. sig: every host value the captured launches depend on
  // (device pointers, forms, solver options); a changed signature drops them.
  struct CgGraph {
    int o = 0, L = 0;
    hipGraphExec_t exec = nullptr;
  };
  std::vector<CgGraph> graphs;
  // Captured per-LM-step sequences (same signature as the CG runs): kind 0 the
  // step prologue (damping, preconditioner, Schur right-hand side, CG start),
  // kind 1 the back-substitution
  struct SeqGraph {
    int kind = 0;
    hipGraphExec_t exec = nullptr;
  };
  std::vector<SeqGraph> seq_graphs;
  std::vector<uintptr_t> graph_sig;
  bool graphs_broken = false;  // a capture failed: eager launches from then on
  const void* graph_comm = nullptr;  // the library communicator whose collectives the graphs hold
  hipEvent_t ev[2] = {nullptr, nullptr};  // the merged LM step's candidate-evaluation span
  hipEvent_t ev_cg[2] = {nullptr, nullptr};  // the CG's pipelined batches
  void drop_graphs() {
    for (CgGraph& g : graphs)
      if (g.exec) (void)hipGraphExecDestroy(g.exec);
    graphs.clear();
    for (SeqGraph& g : seq_graphs)
      if (g.exec) (void)hipGraphExecDestroy(g.exec);
    seq_graphs.clear();
  }
};

// Solver states whose captured graphs hold a library communicator's
// collectives, by communicator (mvba_drop_comm_graphs)
static std::mutex g_comm_graphs_m;
static std::vector<SolverState*> g_comm_graphs;

static void comm_graphs_forget(SolverState* S) {
  std::lock_guard<std::mutex> lk(g_comm_graphs_m);
  g_comm_graphs.erase(std::remove(g_comm_graphs.begin(), g_comm_graphs.end(), S), g_comm_graphs.end());
  S->graph_comm = nullptr;
}

void mvba_drop_comm_graphs(const void* comm) {
  std::lock_guard<std::mutex> lk(g_comm_graphs_m);
  for (SolverState* S : g_comm_graphs)
    if (S->graph_comm == comm) {
      S->drop_graphs();
      S->graph_sig.clear();  // the next solve captures afresh
      S->graph_comm = nullptr;
    }
  g_comm_graphs.erase(std::remove_if(g_comm_graphs.begin(), g_comm_graphs.end(),
                                     [](SolverState* S) { return S->graph_comm == nullptr; }),
                      g_comm_graphs.end());
}

void solver_state_free(SolverState* S) {
  if (!S) return;
  comm_graphs_forget(S);
  S->drop_graphs();  // before the buffers their launches name
  void* ptrs[] = {S->lin, S->phess, S->G, S->cdiag, S->sc, S->dmp, S->fac, S->x, S->xn, S->delta, S->scr, S->lo,
                  S->hi, S->b, S->r, S->r2, S->z, S->p, S->p2, S->q, S->tmp, S->yrep, S->dir, S->dirz, S->dirp[0], S->dirp[1], S->zbuf, S->wbuf, S->cbuf, S->cbuf2, S->obsX, S->du, S->dcbuf,
                  S->cnt, S->partial, S->scal, S->bsize, S->ent, S->goff, S->hoff, S->cam_poff, S->ctl, S->ctl0, S->prec};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (S->hscal) (void)hipHostFree(S->hscal);
  if (S->hctl) (void)hipHostFree(S->hctl);
  if (S->hmir) (void)hipHostFree(S->hmir);
  S->b_det.release();
  S->drop_graphs();
  for (hipEvent_t e : S->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : S->ev_cg)
    if (e) (void)hipEventDestroy(e);
  delete S;
}

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct HipErr {
  hipError_t e;
  const char* where;
};

#define HCHK(x)                                   \
  do {                                            \
    hipError_t e_ = (x);                          \
    if (e_ != hipSuccess) throw HipErr{e_, #x};   \
  } while (0)

struct StatusErr {
  mvba_status st;
  std::string msg;
};

SolverState* alloc_state(mvba_handle* h) {
  SolverState* S = new SolverState();
  S->ng = h->cam_grad_size;
  S->nh = h->cam_hess_size;
  S->np = h->npts;
  S->nc = S->ng + 3 * S->np;
  S->nblocks = (int32_t)h->cam_block_ids.size();
  const int64_t N = h->nres;
  const int64_t ng1 = std::max<int64_t>(S->ng, 1);
  try {
    HCHK(dalloc(&S->lin, (size_t)(S->ng + S->nh + 1)));
    HCHK(dalloc(&S->phess, (size_t)(6 * S->np)));
    for (double** v : {&S->G, &S->cdiag, &S->sc, &S->dmp, &S->x, &S->xn, &S->delta, &S->scr})
      HCHK(dalloc(v, (size_t)S->nc));
    HCHK(dalloc(&S->fac, (size_t)S->nh));
    // q and tmp: one more entry for the exchanged x.y of a sharded solve
    for (double** v : {&S->b, &S->r, &S->r2, &S->z, &S->p, &S->p2}) HCHK(dalloc(v, (size_t)ng1));
    for (double** v : {&S->q, &S->tmp}) HCHK(dalloc(v, (size_t)ng1 + 1));
    const size_t nrep = (size_t)mvba_solver_vec_replicas() * (size_t)ng1;
    HCHK(dalloc(&S->yrep, nrep));
    HCHK(hipMemset(S->yrep, 0, nrep * sizeof(double)));
    HCHK(dalloc(&S->dir, (size_t)(h->nframes * mvba_solver_dir_stride())));
    for (double** v : {&S->dirz, &S->dirp[0], &S->dirp[1]})
      HCHK(dalloc(v, (size_t)(h->nframes * mvba_solver_dir_stride())));
    HCHK(dalloc(&S->prec, (size_t)(h->nframes * mvba::kProjDoubles)));
    HCHK(dalloc(&S->zbuf, (size_t)(8 * N)));
    HCHK(dalloc(&S->wbuf, (size_t)(4 * std::max<int64_t>(S->np, 1))));
    HCHK(dalloc(&S->cbuf, (size_t)(4 * std::max<int64_t>(std::max<int64_t>(N, h->nslots), 1))));
    HCHK(dalloc(&S->cbuf2, (size_t)(2 * std::max<int64_t>(std::max<int64_t>(N, h->nslots), 1))));
    HCHK(dalloc(&S->obsX, (size_t)(4 * std::max<int64_t>(h->nslots, 1))));
    HCHK(dalloc(&S->du, (size_t)(3 * h->ndep_slots)));
    HCHK(dalloc(&S->dcbuf, (size_t)(4 * std::max<int64_t>(h->ndep, 1))));
    HCHK(dalloc(&S->cnt, 8));
    HCHK(hipMemset(S->cnt, 0, 8 * sizeof(unsigned)));
    int64_t ncost = 0;
    for (const Group& G : h->groups) ncost = std::max<int64_t>(ncost, (G.seg_count + 3) / 4);
    // k_cg_update: 3 partials per 256-entry block; k_vec_rep_reduce / k_add_diag one
    S->npartial = std::max<int64_t>({3072, 3 * ((S->ng + 255) / 256), S->ng + 1, mvba_pass_a_blocks(S->np), ncost,
                                    (h->nsegs + 3) / 4,
                                    (int64_t)h->ndep_segs, (h->ndep_slots + 255) / 256}) +
                   1024;  // mvba_launch_sum's second level sits behind the first's partials
    HCHK(dalloc(&S->partial, (size_t)S->npartial));
    HCHK(dalloc(&S->scal, 32));
    HCHK(hipHostMalloc(reinterpret_cast<void**>(&S->hscal), 32 * sizeof(double)));
    HCHK(hipMalloc(reinterpret_cast<void**>(&S->ctl), sizeof(mvba::CgCtl)));
    HCHK(hipMalloc(reinterpret_cast<void**>(&S->ctl0), sizeof(mvba::CgCtl)));
    // [0]: the solve's initial control block (H2D source); [1], [2]: the
    // pipelined batches' read-backs
    HCHK(hipHostMalloc(reinterpret_cast<void**>(&S->hctl), 3 * sizeof(mvba::CgCtl)));
    // (no host-coherent mapped memory: the CG batches end with the copy and the event)
    if (hipHostMalloc(reinterpret_cast<void**>(&S->hmir), sizeof(mvba::CgMirror),
                      hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&S->dmir), S->hmir, 0) != hipSuccess) {
      (void)hipGetLastError();
      if (S->hmir) (void)hipHostFree(S->hmir);
      S->hmir = nullptr;
      S->dmir = nullptr;
    }
    std::vector<int32_t> bs(S->nblocks);
    for (int32_t k = 0; k < S->nblocks; k++) {
      const int32_t bid = h->cam_block_ids[k];
      const int64_t next = (k + 1 < S->nblocks) ? h->cam_goff[k + 1] : S->ng;
      (void)bid;
      bs[k] = (int32_t)(next - h->cam_goff[k]);
    }
    HCHK(upload(&S->bsize, bs));
    std::vector<mvba::CgEntry> em((size_t)S->ng);
    for (int32_t k = 0; k < S->nblocks; k++) {
      S->max_bsize = std::max(S->max_bsize, bs[k]);
      for (int32_t e = 0; e < bs[k]; e++)
        em[(size_t)(h->cam_goff[k] + e)] = {(int32_t)h->cam_goff[k], bs[k], h->cam_hoff[k] + (int64_t)e * bs[k]};
    }
    HCHK(upload(&S->ent, em));
    HCHK(upload(&S->goff, h->cam_goff));
    HCHK(upload(&S->hoff, h->cam_hoff));
    HCHK(upload(&S->cam_poff, h->cam_poff));
    for (hipEvent_t& e : S->ev) HCHK(hipEventCreate(&e));
    for (hipEvent_t& e : S->ev_cg) HCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  } catch (...) {
    solver_state_free(S);
    throw;
  }
  return S;
}

class Solver {
 public:
  Solver(mvba_handle* h, const mvba_solver_options& o, hipStream_t s) : h_(h), o_(o), s_(s), S_(h->solver) {
    flags_ = o.use_loss ? MVBA_EVAL_APPLY_LOSS : 0;
    cauchy_c_ = o.use_loss ? 1.0 / (o.robust_threshold * o.robust_threshold) : 0.0;
    single_model_ = h->groups.size() == 1;
    // the library's own communicators know this rank (fold mode in
    // reduce_frames); a caller's callback does not. MVBA_CG_FOLD=0 keeps the
    // k_add_diag step after the exchange, for A/B timing.
    static const bool no_fold = std::getenv("MVBA_CG_FOLD") && std::getenv("MVBA_CG_FOLD")[0] == '0';
    if (o.allreduce == &mvba_comm_allreduce && !no_fold)
      exch_rank_ = mvba_comm_rank((const mvba_comm*)o.allreduce_user);
    // an RCCL communicator's exchange is one ncclAllReduce on s_: a CG run
    // holding it can be captured like a single-rank one (the local
    // communicator meets its peer threads on the host: eager)
    exch_capturable_ = !o.allreduce || (o.allreduce == &mvba_comm_allreduce &&
                                        mvba_comm_capturable((const mvba_comm*)o.allreduce_user));
  }

  void run(mvba_solver_summary* sum);
  // the frame-order passes' per-slot records (null with MVBA_NO_OBSX=1)
  double4* obsx_records() const { return const_cast<double4*>(obsx()); }

 private:
  mvba_handle* h_;
  const mvba_solver_options& o_;
  hipStream_t s_;
  SolverState* S_;
  int32_t flags_;
  double cauchy_c_;
  bool single_model_;
  bool bounded_ = false;
  int last_cg_iters_ = 0;  // CG iterations of the previous linear solve (batch sizing only)
  int graph_launches_ = 0;  // captured CG runs replayed in this solve (summary)
  // MVBA_CG_TIMING=1: host-side split of the linear-solver wall time, printed
  // at the end of the solve (where a CG iteration's wall time goes)
  struct CgTiming {
    double rhs = 0, start = 0, enqueue = 0, wait = 0, backsub = 0;
    int solves = 0, batches = 0, enqueued = 0, iters = 0;
  } tm_;
  static bool cg_timing() {
    static const bool on = std::getenv("MVBA_CG_TIMING") && std::getenv("MVBA_CG_TIMING")[0] == '1';
    return on;
  }
  int32_t exch_rank_ = -1;  // this rank, when the exchange is a library communicator
  bool exch_capturable_ = true;  // no exchange, or one a stream capture can hold (RCCL)
  // Single-rank, non-deterministic CG: the replica reduction adds p.q into
  // scal[kPqSlot + par] with one atomic per block (no finalising block) and the
  // update kernel takes the step length from it; par = the CG iteration's
  // parity (double buffer: each reduction zeroes the slot the previous update
  // read). MVBA_CG_PQ=grid keeps the last-block reduction (A/B timing).
  static constexpr int kPqSlot = 24;
  int cg_par_ = 0;
  bool merged_reads() const {
    const char* e = std::getenv("MVBA_LM_MERGED");  // read per call: tests switch it
    return !(e && e[0] == '0');
  }
  bool pq_atomic() const {
    const char* e = std::getenv("MVBA_CG_PQ");  // read per call: tests switch it
    return !o_.allreduce && !o_.deterministic && !(e && !std::strcmp(e, "grid"));
  }

  int pa_model() const { return single_model_ ? h_->groups[0].model : -1; }
  // per-slot landmark copy for the frame-order passes (MVBA_NO_OBSX=1: gather
  // through obs_pid as before, for A/B timing)
  const double4* obsx() const {
    static const bool off = std::getenv("MVBA_NO_OBSX") && std::getenv("MVBA_NO_OBSX")[0] == '1';
    return off ? nullptr : (const double4*)S_->obsX;
  }
  int pa_deg() const { return single_model_ ? h_->groups[0].deg : 0; }

  // Cross-rank sum / max of a device buffer, stream-ordered (mvba_allreduce_fn:
  // enqueued on s_, no host wait here).
  void exchange(double* buf, int64_t n, int32_t op) {
    if (!o_.allreduce || n <= 0) return;
    if (o_.allreduce(buf, n, op, (void*)s_, o_.allreduce_user) != 0)
      throw StatusErr{MVBA_E_INVALID, "allreduce callback failed"};
  }

  // Fetch device scalars scal[0..n) to the pinned mirror (one sync).
  const double* fetch(int n) {
    HCHK(hipMemcpyAsync(S_->hscal, S_->scal, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s_));
    HCHK(hipStreamSynchronize(s_));
    return S_->hscal;
  }

  void dot(int64_t n, const double* a, const double* b, int slot) {
    HCHK(mvba_launch_dot(n, a, b, S_->partial, S_->cnt + 6, S_->scal + slot, s_));
  }

  void prep() {
    h_->gen++;
    HCHK(mvba_launch_prep(h_->d_fd, h_->nframes, h_->d_params, h_->d_frec, h_->d_pt_off, h_->d_pt_free, h_->npts,
                          h_->d_pts, h_->gen, h_->d_err, s_));
    h_->prep_done = true;
  }

  void check_alpha() {
    HCHK(hipStreamSynchronize(s_));
    int err[2] = {0, 0};
    HCHK(hipMemcpy(err, h_->d_err, sizeof(err), hipMemcpyDeviceToHost));
    const mvba_status st = device_error(err, h_->gen);
    if (st != MVBA_OK) throw StatusErr{st, device_error_text(st)};
  }

  // Jacobian at the handle's parameters -> lin (all-reduced), G, phess, cdiag. Returns cost.
  // skip_prep: the frame and landmark records are current (the candidate's
  // cost evaluation just ran the prep kernel at these parameters)
  // enqueue-only form (merged LM step): the cost lands in scal[cost_slot], the
  // device error word is read with the step's one fetch (fetch_checked)
  void linearize_enqueue(bool skip_prep, int cost_slot) {
    const int32_t lf = flags_ | (o_.deterministic ? MVBA_LIN_DETERMINISTIC : 0) | (skip_prep ? MVBA_EVAL_SKIP_PREP : 0);
    mvba_status st = mvba_linearize_device(h_, lf, o_.robust_threshold, S_->lin, S_->lin + S_->ng,
                                           S_->G + S_->ng, S_->phess, S_->lin + S_->ng + S_->nh, (void*)s_);
    if (st != MVBA_OK) throw StatusErr{st, h_->err};
    exchange(S_->lin, S_->ng + S_->nh + 1, MVBA_REDUCE_SUM);
    if (S_->ng)
      HCHK(hipMemcpyAsync(S_->G, S_->lin, (size_t)S_->ng * sizeof(double), hipMemcpyDeviceToDevice, s_));
    HCHK(mvba_launch_extract_diag(S_->nblocks, S_->goff, S_->hoff, S_->bsize, S_->lin + S_->ng, S_->np, S_->phess,
                                  S_->ng, S_->cdiag, s_));
    HCHK(hipMemcpyAsync(S_->scal + cost_slot, S_->lin + S_->ng + S_->nh, sizeof(double), hipMemcpyDeviceToDevice,
                        s_));
  }
  void grad_max_enqueue(int slot) {
    HCHK(mvba_launch_proj_grad_max(S_->nc, S_->x, S_->G, S_->lo, S_->hi, S_->partial, S_->scal + slot, s_));
    exchange(S_->scal + slot, 1, MVBA_REDUCE_MAX);
  }

  double linearize(bool skip_prep = false) {
    const int32_t lf = flags_ | (o_.deterministic ? MVBA_LIN_DETERMINISTIC : 0) | (skip_prep ? MVBA_EVAL_SKIP_PREP : 0);
    mvba_status st = mvba_linearize_device(h_, lf, o_.robust_threshold, S_->lin, S_->lin + S_->ng,
                                           S_->G + S_->ng, S_->phess, S_->lin + S_->ng + S_->nh, (void*)s_);
    if (st != MVBA_OK) throw StatusErr{st, h_->err};
    check_alpha();
    exchange(S_->lin, S_->ng + S_->nh + 1, MVBA_REDUCE_SUM);
    if (S_->ng)
      HCHK(hipMemcpyAsync(S_->G, S_->lin, (size_t)S_->ng * sizeof(double), hipMemcpyDeviceToDevice, s_));
    HCHK(mvba_launch_extract_diag(S_->nblocks, S_->goff, S_->hoff, S_->bsize, S_->lin + S_->ng, S_->np, S_->phess,
                                  S_->ng, S_->cdiag, s_));
    double c = 0.0;
    HCHK(hipMemcpyAsync(&c, S_->lin + S_->ng + S_->nh, sizeof(double), hipMemcpyDeviceToHost, s_));
    HCHK(hipStreamSynchronize(s_));
    return c;
  }

  // One host read of scal[0..n) and the device error word (K0's alpha range
  // check); throws on a device error. The merged LM step below reads every
  // scalar a decision needs with one of these instead of one sync per quantity.
  // deferred: the device error is returned there instead of thrown (the merged
  // step's candidate evaluation, whose error counts only for a valid step)
  const double* fetch_checked(int n, mvba_status* deferred = nullptr) {
    HCHK(hipMemcpyAsync(S_->hscal, S_->scal, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s_));
    HCHK(hipMemcpyAsync(S_->hscal + kErrSlot, h_->d_err, 2 * sizeof(int), hipMemcpyDeviceToHost, s_));
    HCHK(hipStreamSynchronize(s_));
    int err[2];
    std::memcpy(err, S_->hscal + kErrSlot, sizeof(err));
    const mvba_status st = device_error(err, h_->gen);
    if (deferred)
      *deferred = st;
    else if (st != MVBA_OK)
      throw StatusErr{st, device_error_text(st)};
    return S_->hscal;
  }
  static constexpr int kErrSlot = 30;  // hscal[30]: the device error word (2 ints)

  // cost() without its host reads: the candidate's cost into scal[16], summed
  // over ranks (stream-ordered)
  void cost_enqueue() {
    prep();
    double* acc = S_->scal + 16;
    HCHK(hipMemsetAsync(acc, 0, sizeof(double), s_));
    for (const Group& G : h_->groups) {
      int64_t nb = 0;
      HCHK(mvba_launch_cost(G.model, G.deg, h_->d_segs + G.seg_begin, G.seg_count, h_->d_fd, h_->d_frec,
                            h_->d_params, h_->d_pts, h_->d_obs_pid, h_->d_obs_meas, flags_, cauchy_c_,
                            S_->partial, s_, &nb));
      HCHK(mvba_launch_sum(nb, S_->partial, S_->scal + 17, s_));
      HCHK(mvba_launch_axpby(1, 1.0, acc, 1.0, S_->scal + 17, acc, s_));
    }
    if (h_->ndep > 0) {
      int64_t nb = 0;
      HCHK(mvba_launch_depth_cost(h_->ndep_slots, h_->d_dep_desc, h_->d_dep_order, h_->d_dep_meas, h_->d_frec,
                                  h_->d_params, h_->d_pts, flags_, cauchy_c_, S_->partial, s_, &nb));
      HCHK(mvba_launch_sum(nb, S_->partial, S_->scal + 17, s_));
      HCHK(mvba_launch_axpby(1, 1.0, acc, 1.0, S_->scal + 17, acc, s_));
    }
    if (h_->nxyz > 0) {
      HCHK(mvba_launch_xyz_cost(h_->nxyz, h_->d_xpid, h_->d_xref, h_->d_xcc, h_->d_pts, flags_, h_->d_xscal + 1,
                                h_->d_xcnt, h_->d_xscal, s_));
      HCHK(mvba_launch_axpby(1, 1.0, acc, 1.0, h_->d_xscal, acc, s_));
    }
    exchange(acc, 1, MVBA_REDUCE_SUM);
  }

  // |v|^2 over the compact vector into scal[pt_slot] (points, summed over
  // ranks) and scal[cam_slot] (camera part, replicated), no host read
  void norm2_enqueue(const double* v, int pt_slot, int cam_slot) {
    dot(3 * S_->np, v + S_->ng, v + S_->ng, pt_slot);
    exchange(S_->scal + pt_slot, 1, MVBA_REDUCE_SUM);
    dot(S_->ng, v, v, cam_slot);
  }

  // Cost at the handle's parameters (prep + cost kernels), summed over ranks.
  double cost() {
    prep();
    double* acc = S_->scal + 16;
    HCHK(hipMemsetAsync(acc, 0, sizeof(double), s_));
    for (const Group& G : h_->groups) {
      int64_t nb = 0;
      HCHK(mvba_launch_cost(G.model, G.deg, h_->d_segs + G.seg_begin, G.seg_count, h_->d_fd, h_->d_frec,
                            h_->d_params, h_->d_pts, h_->d_obs_pid, h_->d_obs_meas, flags_, cauchy_c_,
                            S_->partial, s_, &nb));
      HCHK(mvba_launch_sum(nb, S_->partial, S_->scal + 17, s_));
      HCHK(mvba_launch_axpby(1, 1.0, acc, 1.0, S_->scal + 17, acc, s_));
    }
    if (h_->ndep > 0) {
      int64_t nb = 0;
      HCHK(mvba_launch_depth_cost(h_->ndep_slots, h_->d_dep_desc, h_->d_dep_order, h_->d_dep_meas, h_->d_frec,
                                  h_->d_params, h_->d_pts, flags_, cauchy_c_, S_->partial, s_, &nb));
      HCHK(mvba_launch_sum(nb, S_->partial, S_->scal + 17, s_));
      HCHK(mvba_launch_axpby(1, 1.0, acc, 1.0, S_->scal + 17, acc, s_));
    }
    if (h_->nxyz > 0) {
      HCHK(mvba_launch_xyz_cost(h_->nxyz, h_->d_xpid, h_->d_xref, h_->d_xcc, h_->d_pts, flags_, h_->d_xscal + 1,
                                h_->d_xcnt, h_->d_xscal, s_));
      HCHK(mvba_launch_axpby(1, 1.0, acc, 1.0, h_->d_xscal, acc, s_));
    }
    check_alpha();
    exchange(acc, 1, MVBA_REDUCE_SUM);
    HCHK(hipMemcpyAsync(S_->hscal + 16, acc, sizeof(double), hipMemcpyDeviceToHost, s_));
    HCHK(hipStreamSynchronize(s_));
    return S_->hscal[16];
  }

  // pass B over every model group into the replicas, then y = sum of replicas.
  // Single rank: damping and the x.y dot are fused into the replica reduction
  // (dot -> scal[dot_slot]); sharded: cross-rank sum of y first (stream-ordered),
  // then damping + dot. gate: device CG stop flag (nullptr: always run); ctl:
  // CG step-length logic in the finalising block of the x.y reduction
  // dir: the frame directions of xv (null: pass B with x = 0, u_o = -J_pt w_p);
  // lz: xv is the CG direction, formed (and stored) by the reduction that damps it
  void reduce_frames(double* y, const double* xv, int dot_slot, const double* dir, const int32_t* gate = nullptr,
                     mvba::CgCtl* ctl = nullptr, const mvba::LazyDir* lz = nullptr) {
    // deterministic mode: slab rows per chunk / depth segment and a fixed-order
    // gather instead of replica atomics (the first product records the plan)
    DetPlan& D = S_->b_det;
    const bool det = o_.deterministic != 0;
    if (det && !D.ready)
      HCHK(det_plan_begin(D, (int64_t)h_->nchunks + h_->ndep_segs, mvba::vec_slab_width(h_->kmax), S_->ng, s_));
    for (const Group& G : h_->groups)
      HCHK(mvba_launch_pass_b(G.model, G.deg, h_->d_chunks + G.chunk_begin, G.chunk_count, G.chunk_begin,
                              h_->d_segs, h_->d_fd, h_->d_frame_lin, h_->d_frec, h_->d_params, h_->d_pts,
                              h_->d_obs_pid, h_->d_obs_meas, dir, (const double4*)S_->wbuf, S_->yrep, S_->ng, flags_,
                              cauchy_c_, gate, det ? D.slab(0) : no_slab(), obsx(), s_));
    if (h_->ndep > 0)
      HCHK(mvba_launch_depth_sb(h_->d_dep_segs, h_->ndep_segs, h_->d_dep_desc, h_->d_dep_pid, h_->d_dep_meas, h_->d_frec,
                                h_->d_params, h_->d_pts, h_->d_frame_lin, S_->du, S_->yrep, S_->ng, flags_, cauchy_c_,
                                gate, det ? D.slab(h_->nchunks) : no_slab(),
                                dir ? (const double4*)S_->wbuf : nullptr, s_));  // dir: du holds z_d (k_depth_pa)
    if (det && !D.ready) HCHK(det_plan_finish(D, s_));
    // fuse (single rank): damping, x.y and the step length in the reduction.
    // fold (sharded, library communicator: the rank is known): rank 0 adds the
    // damping D x to its share, every rank appends its share of x.y to y, the
    // exchange sums both, and the update kernel takes the step length from the
    // summed dot (pq_of). Otherwise (a caller's own all-reduce) the damping and
    // the dot follow the exchange in k_add_diag.
    const bool fuse = xv && !o_.allreduce;
    const bool fold = xv && o_.allreduce && exch_rank_ >= 0;
    const bool any = fuse || fold;
    const bool atomic_pq = fuse && ctl && !det && pq_atomic();
    const double* dg = (fuse || (fold && exch_rank_ == 0)) ? S_->dmp : nullptr;
    double* dot_out = atomic_pq ? S_->scal + kPqSlot + cg_par_
                      : fuse   ? S_->scal + dot_slot
                      : fold   ? y + S_->ng
                               : nullptr;
    if (det)
      HCHK(mvba_launch_slab_reduce_vec(D.tier_view(), D.grid(), D.begin, D.pos, D.val, dg, any ? xv : nullptr, y,
                                       S_->partial, S_->cnt + 4, dot_out, gate, any ? ctl : nullptr,
                                       any ? lz : nullptr, fold ? 1 : 0, s_));
    else
      HCHK(mvba_launch_rep_reduce_vec(S_->yrep, S_->ng, dg, any ? xv : nullptr, y, S_->partial, S_->cnt + 4, dot_out,
                                      gate, any ? ctl : nullptr, any ? lz : nullptr, atomic_pq ? 2 : fold ? 1 : 0,
                                      S_->scal + kPqSlot + (cg_par_ ^ 1), s_));
    exchange(y, S_->ng + (fold ? 1 : 0), MVBA_REDUCE_SUM);
    if (xv && !any)
      HCHK(mvba_launch_add_diag(S_->ng, S_->dmp, xv, y, S_->partial, S_->cnt + 4, S_->scal + dot_slot, gate, ctl,
                                lz, s_));
  }
  // the exchanged p.q behind a product vector q (fold mode), else null
  // (fold mode), or the CG product's atomic accumulator (single rank), else null
  const double* pq_of(const double* q) const {
    if (o_.allreduce && exch_rank_ >= 0) return q + S_->ng;
    if (q == S_->q && pq_atomic()) return S_->scal + kPqSlot + cg_par_;
    return nullptr;
  }

  static mvba::DirPair plain_dir(const double* dir) { return mvba::DirPair{dir, nullptr, nullptr, nullptr}; }

  // Where pass A leaves c_o: slot order (coalesced stores, k_point_w gathers).
  // With frames in first-use order the point-order scatter won below ~128 MB of
  // table (profiles/r03/ab_co_order/: c2 pass A + k_point_w 29.8 us point order
  // vs 36.0 slot order; c3 395 vs 327 us); with frames in capture order (the
  // gathers of neighbouring landmarks share lines) slot order wins at both
  // sizes (profiles/r04/r04m/: c2 27.9 vs 29.0 us, c3 303 vs 361 us).
  // MVBA_CO_ORDER=point|slot forces one.
  bool co_slot_order(const char* env) const {
    return !(env && !std::strcmp(env, "point"));
  }

  // w_p = (V + D)^-1 (tinit + sum J_pt^T J_cam x) into wbuf (dr: frame
  // directions of x, dr.dz null for x = 0). Depth blocks need the point-lane kernel
  // (it also forms their u_d); otherwise the frame-order sweep + point solve.
  void pass_a_w(const mvba::DirPair& dr, const double* tinit, const double* xv, const int32_t* gate) {
    // x != 0: frame records given (dz), or formed by pass A from z (frec)
    const double* dir = dr.dz ? dr.dz : dr.frec;
    if (h_->ndep > 0 && !dir) {
      // right-hand side (x = 0): the point-order kernel also forms u_d = -P w_p
      HCHK(mvba_launch_pass_a(pa_model(), pa_deg(), h_->d_pt_begin, h_->npts, h_->d_po_frame, h_->d_po_meas,
                              h_->d_fd, h_->d_frec, h_->d_params, h_->d_pts, dir, tinit, S_->phess,
                              S_->dmp + S_->ng, S_->zbuf, S_->wbuf, 4, nullptr, nullptr, nullptr, flags_, cauchy_c_,
                              h_->point_extra(), xv, S_->du, gate, S_->prec, s_));
      return;
    }
    // one chunk of up to 8 segments of one image per wave (d_achunks; pass B's
    // chunks are 16 segments where images average 12+) when there are
    // enough of them to fill the chip (4,096+, four waves per SIMD): with frames
    // in capture order the landmark gathers are cheap and the direction staging
    // per wave amortises over more observations (c3, 18k chunks: pass A 176 ->
    // 132-144 us; c2, 3k chunks: equal; a 1/8 c2 shard, 470 chunks: 6.0 -> 10.3
    // us, so it keeps one segment per wave; profiles/r04/r04t/, r04w/).
    // MVBA_PASS_A_CHUNKS=0|1 forces one (read per call, for A/B timing)
    const bool chunked = pass_a_chunked();
    // where pass A leaves c_o = J_pt^T z_o: at the observation's point-order
    // position (scattered 32-B stores, k_point_w reads its run) or in slot order
    // (coalesced stores, k_point_w gathers through po_slot). MVBA_CO_ORDER=
    // point|slot forces one, for A/B timing.
    const char* co_env = std::getenv("MVBA_CO_ORDER");  // read per call: tests switch it
    const bool co_slot = co_slot_order(co_env);
    if (dir)
      for (const Group& G : h_->groups)
        HCHK(mvba_launch_pass_a_frame(G.model, G.deg,
                                      chunked ? h_->d_achunks + G.achunk_begin : h_->d_segchunks + G.seg_begin,
                                      chunked ? G.achunk_count : G.seg_count, h_->d_segs,
                                      h_->d_pts, h_->d_obs_pid, h_->d_obs_meas, co_slot ? nullptr : h_->d_slot_po, dr,
                                      (double4*)S_->cbuf, flags_, cauchy_c_, gate, S_->prec, obsx(), s_));
    // depth blocks in frame order (z_d into du, P z_d per block for the point solve)
    // (depth problems never take the pass-A-formed records: fused_dir is off)
    const bool dep = dr.dz && h_->ndep > 0;
    if (dep)
      HCHK(mvba_launch_depth_pa(h_->d_dep_segs, h_->ndep_segs, h_->d_dep_desc, h_->d_dep_pid, h_->d_dep_meas,
                                h_->d_frec, h_->d_params, h_->d_pts, dr.dz, xv, S_->du, h_->d_dslot_po,
                                (double4*)S_->dcbuf, flags_, cauchy_c_, gate, s_));
    if (dir && !dep && point_w_tiles())
      HCHK(mvba_launch_point_w_seg(h_->nwtiles, h_->d_wtiles, h_->d_wlane_pid,
                                   co_slot ? h_->d_wlane_slot : h_->d_wlane_pos, h_->d_pt_begin,
                                   co_slot ? h_->d_po_slot : nullptr, (const double4*)S_->cbuf, tinit, S_->phess,
                                   S_->dmp + S_->ng, h_->d_pts, S_->wbuf, 4, gate, s_));
    else
      HCHK(mvba_launch_point_w(h_->npts, h_->d_pt_begin, co_slot ? h_->d_po_slot : nullptr,
                               dir ? (const double4*)S_->cbuf : nullptr,
                               tinit, S_->phess, S_->dmp + S_->ng, h_->d_pts, S_->wbuf, 4, gate,
                               dep ? h_->d_dpt_begin : nullptr, dep ? (const double4*)S_->dcbuf : nullptr, nullptr,
                               s_));
  }

  bool pass_a_chunked() const {
    const char* pa_env = std::getenv("MVBA_PASS_A_CHUNKS");
    int32_t nchunks_all = 0;
    for (const Group& G : h_->groups) nchunks_all += G.achunk_count;
    return pa_env ? pa_env[0] == '1' : nchunks_all >= 4096;
  }

  // The fused CG step (k_upd_pass_a, mvba::FusedStep): the update of
  // iteration i - 1 runs in the launch of iteration i's pass A, one grid-wide
  // phase per CG iteration less; pass A then stores two products (+16 B per
  // observation each way through k_point_w), which pays where the phases'
  // fixed latency dominates: thin shards. Reprojection-only problems of one
  // model group with the frame records from the update (fused_dir, not
  // MVBA_CG_DZ=passa), per-slot records and the lane point solve.
  // MVBA_CG_FUSE=0|1 forces it off / on (read per call); by default it runs
  // below kFuseMaxObs observations.
  static constexpr int64_t kFuseMaxObs = 400000;
  bool fused_step() const {
    if (!fused_dir() || dz_in_pass_a() || h_->groups.size() != 1 || !obsx() || point_w_tiles()) return false;
    const char* e = std::getenv("MVBA_CG_FUSE");
    if (e) return e[0] == '1';
    return h_->nres <= kFuseMaxObs;
  }

  // k_point_w_seg (wave tiles of whole tracks, one lane per residual) when
  // MVBA_POINT_W=tiles; the default is 8 lanes per point (k_point_w)
  bool point_w_tiles() const {
    const char* e = std::getenv("MVBA_POINT_W");  // read per call: tests switch it
    return h_->nwtiles > 0 && e && !std::strcmp(e, "tiles");
  }

  // y = S x (implicit Schur complement with damping); x.y -> scal[dot_slot].
  // lz: x is the CG direction formed by the frame-direction kernel (into xv)
  void apply_schur(const double* xv, double* y, int dot_slot, const int32_t* gate = nullptr,
                   mvba::CgCtl* ctl = nullptr, const mvba::LazyDir* lz = nullptr) {
    HCHK(mvba_launch_frame_dir(h_->d_frame_lin, (int32_t)h_->nframes, h_->d_fd, h_->d_frec, xv, S_->dir, gate, lz,
                               s_));
    pass_a_w(plain_dir(S_->dir), nullptr, xv, gate);
    reduce_frames(y, xv, dot_slot, S_->dir, gate, ctl);
  }

  // y = S p_new for the CG direction p_new = z (+ beta p_old) with no direction
  // kernel: pass A forms the frame records dz + beta dp (dz = W z, written by the
  // CG update's frame blocks; dp = the previous product's, DirPair) and keeps
  // them in dr.dp_out, which pass B then reads; p_new itself is formed by the
  // reduction that damps it (lz). Reprojection-only problems.
  void apply_schur_cg(double* y, const int32_t* gate, mvba::CgCtl* ctl, const mvba::LazyDir& lz,
                      const mvba::DirPair& dr) {
    pass_a_w(dr, nullptr, lz.p_new, gate);
    reduce_frames(y, lz.p_new, 0, dr.dp_out, gate, ctl, &lz);
  }

  // b = -(g_c - W (V+D)^-1 g_p). Starts every linear solve: the projection
  // records for pass A are built here (parameters fixed until the next step).
  void schur_rhs() {
    HCHK(mvba_launch_frame_proj((int32_t)h_->nframes, h_->d_fd, h_->d_frec, h_->d_params, S_->prec, s_));
    pass_a_w(plain_dir(nullptr), S_->G + S_->ng, nullptr, nullptr);
    reduce_frames(S_->tmp, nullptr, 0, nullptr);  // = -W w
    HCHK(mvba_launch_axpby(S_->ng, -1.0, S_->G, -1.0, S_->tmp, S_->b, s_));
  }

  struct CgResult {
    int iters = 0;
    int status = 0;  // 0 success, 1 no convergence (usable), 2 failure
  };

  // PCG on S delta_c = b (conjugate_gradients_solver.cc [ext]) with every
  // scalar step on the device (CgCtl): iterations are enqueued in batches and
  // gated by ctl->done, one host read per batch. Sharded solves run the same
  // loop: the per-iteration exchange of the product is stream-ordered and the
  // replicated camera-side state gives every rank the same stopping decisions.
  // Host values the launches of one CG iteration depend on, beyond the
  // iteration's offset in the reset period: a captured iteration is replayed
  // only while all of them are unchanged.
  std::vector<uintptr_t> cg_signature(bool fused_dir) const {
    auto u = [](const void* p) { return (uintptr_t)p; };
    // the launch-shaping switches read at enqueue time, by their first character
    auto env0 = [](const char* name) {
      const char* e = std::getenv(name);
      return (uintptr_t)(e ? (unsigned char)e[0] : 0u);
    };
    // an fp64 host value by its exact bit pattern, not a rounding of it
    auto bits = [](double v) {
      uint64_t b = 0;
      static_assert(sizeof(b) == sizeof(v), "fp64 bit pattern");
      std::memcpy(&b, &v, sizeof(b));
      return (uintptr_t)b;
    };
    const char* co = std::getenv("MVBA_CO_ORDER");
    std::vector<uintptr_t> v = {
        (uintptr_t)fused_dir, (uintptr_t)pq_atomic(), (uintptr_t)co_slot_order(co), env0("MVBA_PASS_A_CHUNKS"),
        env0("MVBA_PASSB_WAVES"), (uintptr_t)point_w_tiles(), u(h_->d_wtiles), u(h_->d_wlane_pid),
        u(h_->d_wlane_slot), u(h_->d_wlane_pos), (uintptr_t)flags_, bits(cauchy_c_), (uintptr_t)S_->ng,
        (uintptr_t)h_->nframes, u((const void*)o_.allreduce), u(o_.allreduce_user), (uintptr_t)(intptr_t)exch_rank_,
        u(obsx()), u(h_->d_params), u(h_->d_pts), u(h_->d_frec), u(h_->d_fd), u(h_->d_frame_lin), u(h_->d_segs),
        u(h_->d_chunks), u(h_->d_segchunks), u(h_->d_achunks), u(h_->d_obs_pid), u(h_->d_obs_meas), u(h_->d_slot_po),
        u(h_->d_po_slot), u(h_->d_pt_begin), u(h_->d_pt_off), u(h_->d_pt_free), u(h_->d_dep_segs),
        u(h_->d_dep_desc), u(h_->d_dep_pid), u(h_->d_dep_meas), u(h_->d_dslot_po), u(h_->d_dpt_begin),
        u(h_->d_po_frame), u(h_->d_po_meas), (uintptr_t)h_->npts, (uintptr_t)h_->nchunks,
        (uintptr_t)h_->ndep_segs, (uintptr_t)o_.deterministic,
        // the step prologue and back-substitution graphs (enqueue_seq)
        bits(o_.min_lm_diagonal), bits(o_.max_lm_diagonal), (uintptr_t)o_.jacobi_scaling, env0("MVBA_BACKSUB"), env0("MVBA_CG_DZ"), env0("MVBA_CG_FUSE"), env0("MVBA_REP_THREADS"),
        (uintptr_t)mirror_on(), u(S_->dmir),
        (uintptr_t)h_->ndep, (uintptr_t)h_->nxyz, u(h_->d_dpo_slot), u(h_->d_xpt_begin), u(h_->d_xref), u(h_->d_xcc),
        u(h_->d_dep_order)};
    if (o_.deterministic) {
      const DetPlan& D = S_->b_det;
      for (uintptr_t x : {u(D.val), u(D.begin), u(D.pos), u(D.tiers), (uintptr_t)D.nheavy, (uintptr_t)D.nmedium,
                          (uintptr_t)D.nlight, (uintptr_t)D.width})
        v.push_back(x);
    }
    for (const Group& G : h_->groups) {
      v.push_back((uintptr_t)G.model);
      v.push_back((uintptr_t)G.deg);
      v.push_back((uintptr_t)G.chunk_begin);
      v.push_back((uintptr_t)G.chunk_count);
      v.push_back((uintptr_t)G.seg_begin);
      v.push_back((uintptr_t)G.seg_count);
      v.push_back((uintptr_t)G.achunk_begin);
      v.push_back((uintptr_t)G.achunk_count);
    }
    return v;
  }

  // PCG on S delta_c = b (conjugate_gradients_solver.cc [ext]) with every
  // scalar step on the device (CgCtl): iterations are enqueued in batches and
  // gated by ctl->done, one host read per batch. Sharded solves run the same
  // loop: the per-iteration exchange of the product is stream-ordered and the
  // replicated camera-side state gives every rank the same stopping decisions.
  //
  // Every launch argument of iteration i is a function of i mod 10 (the
  // double-buffered p, r, direction records and p.q accumulator by the parity
  // of i, the residual reset at i % 10 == 0; the iteration number itself is
  // counted on the device, CgCtl::it), so single-rank solves capture runs of
  // iterations as hipGraphs once per handle and replay them (RCCL-sharded
  // solves too, with the exchange inside the graph): a batch of k
  // iterations costs a few graph launches instead of 5 k kernel launches, whose
  // host time (≈ 25 us per iteration, 5-6 us per hipLaunchKernel) bound the
  // CG iteration of small problems (profiles/r05/r05b/s8_timing_r05b.log:
  // enqueue 27.6 us vs 16.1 us of wait per iteration on the 1/8 c2 shard).
  // MVBA_CG_GRAPH=0: eager launches (A/B timing).
  // Reprojection-only problems: the CG update's frame blocks form W z and the
  // products combine it with the previous product's records (no direction
  // kernel per iteration). Depth blocks read the direction in more kernels:
  // they keep the direction kernel (MVBA_CG_DIR_KERNEL=1 forces it, for A/B).
  bool fused_dir() const {
    const char* dk_env = std::getenv("MVBA_CG_DIR_KERNEL");  // read per call: tests switch it
    return h_->ndep == 0 && !(dk_env && dk_env[0] == '1');
  }
  // With fused_dir, MVBA_CG_DZ=passa: pass A forms the pose sums W_f z of its
  // frame from z (stage_dir, DirPair::frec), so the CG update launches its
  // entry blocks only. Measured slower, not the default (kernel traces,
  // profiles/r06/r06a/cg_iter_r06a.txt): the update's time is its entry
  // blocks' grid reduction (1/8 c2 shard 7.28 vs 7.52 us without / with the
  // frame blocks; c2 8.32 vs 9.76), while every pass-A wave pays the frame's
  // W z (a FrameLin load, then the z gathers: pass A 7.36 vs 5.60 us, c2 20.9
  // vs 16.5). Default: the update's frame blocks write dz (read per call).
  bool dz_in_pass_a() const {
    const char* e = std::getenv("MVBA_CG_DZ");  // read per call: tests switch it
    return fused_dir() && e && !std::strcmp(e, "passa");
  }

  // Graphs: single rank, or a sharded solve exchanging through an RCCL
  // communicator (the ncclAllReduce is captured with the kernels around it:
  // every rank replays the same runs, since the replicated camera-side CG state
  // gives every rank the same batches); a caller's callback or the local
  // communicator (host rendezvous) stays eager; a capturable (non-null)
  // stream; deterministic mode once its slab plan is recorded (the first
  // product records it). MVBA_CG_GRAPH=0: eager launches (A/B timing).
  bool graphs_enabled() const {
    const char* g_env = std::getenv("MVBA_CG_GRAPH");  // read per call: tests switch it
    return !(g_env && g_env[0] == '0') && exch_capturable_ && s_ != nullptr &&
           (!o_.deterministic || S_->b_det.ready) && !S_->graphs_broken;
  }
  // CG batches end in a host-coherent CgMirror (cg_device); MVBA_CG_MIRROR=0
  // or pipelined batches (MVBA_CG_PIPE=1): a copy launch and an event
  bool mirror_on() const {
    const char* m = std::getenv("MVBA_CG_MIRROR");  // read per call: tests switch it
    const char* pp = std::getenv("MVBA_CG_PIPE");
    return S_->dmir && !(m && m[0] == '0') && !(pp && pp[0] == '1');
  }
  // drops every captured graph whose launches no longer match (signature)
  void refresh_graph_sig() {
    if (!graphs_enabled()) return;
    std::vector<uintptr_t> sig = cg_signature(fused_dir());
    if (sig != S_->graph_sig) {
      S_->drop_graphs();
      S_->graph_sig = std::move(sig);
    }
  }

  // Captures fn's enqueues on s_ into *exec. A refused capture is reported once
  // per handle (stderr), graphs are off for the handle from then on, and the
  // caller runs fn eagerly: the launches and exchanges of a failed capture
  // never ran, so every rank (which fails the same way) re-enqueues them.
  template <class F>
  bool capture(F&& fn, hipGraphExec_t* exec) {
    *exec = nullptr;
    hipGraph_t graph = nullptr;
    auto broken = [&](const char* what, hipError_t e) {
      (void)hipGetLastError();
      S_->graphs_broken = true;
      std::fprintf(stderr, "mvba_solve: graph capture refused at %s (%s)%s; eager launches from here\n", what,
                   hipGetErrorString(e), o_.allreduce ? " with the RCCL exchange inside" : "");
    };
    const hipError_t eb = hipStreamBeginCapture(s_, hipStreamCaptureModeThreadLocal);
    if (eb != hipSuccess) {
      broken("hipStreamBeginCapture", eb);
      return false;
    }
    bool ok = true;
    try {
      fn();
    } catch (...) {
      ok = false;
    }
    const hipError_t ec = hipStreamEndCapture(s_, &graph);
    hipError_t ei = hipSuccess;
    if (ok && ec == hipSuccess && graph) ei = hipGraphInstantiate(exec, graph, nullptr, nullptr, 0);
    if (graph) (void)hipGraphDestroy(graph);
    if (!ok || ec != hipSuccess || !graph || ei != hipSuccess) {
      if (*exec) (void)hipGraphExecDestroy(*exec);
      *exec = nullptr;
      broken(!ok ? "an enqueue inside the capture" : ec != hipSuccess || !graph ? "hipStreamEndCapture"
                                                                                : "hipGraphInstantiate",
             !ok ? hipErrorStreamCaptureInvalidated : ec != hipSuccess ? ec : ei);
      return false;
    }
    if (o_.allreduce == &mvba_comm_allreduce && S_->graph_comm != o_.allreduce_user) {
      // the graph holds this communicator's collectives: mvba_comm_destroy drops it first
      std::lock_guard<std::mutex> lk(g_comm_graphs_m);
      if (!S_->graph_comm) g_comm_graphs.push_back(S_);
      S_->graph_comm = o_.allreduce_user;
    }
    return true;
  }

  // A per-LM-step sequence (kind: SolverState::SeqGraph): replayed from its
  // captured graph (captured at first use), or enqueued eagerly when graphs are
  // off. fn's launch arguments must be fixed for the signature (the damping's
  // 1/radius is read from device memory for that reason).
  template <class F>
  void enqueue_seq(int kind, F&& fn) {
    if (!graphs_enabled()) {
      fn();
      return;
    }
    for (const SolverState::SeqGraph& g : S_->seq_graphs)
      if (g.kind == kind) {
        HCHK(hipGraphLaunch(g.exec, s_));
        graph_launches_++;
        return;
      }
    hipGraphExec_t exec = nullptr;
    if (!capture(fn, &exec)) {
      fn();
      return;
    }
    S_->seq_graphs.push_back(SolverState::SeqGraph{kind, exec});
    HCHK(hipGraphLaunch(exec, s_));
    graph_launches_++;
  }

  // Start of a linear solve, enqueue only (part of the step prologue): x = 0,
  // the control block from the solve's template, b.b, r = b, z = M^-1 r, rho.
  void cg_start() {
    const int64_t n = S_->ng;
    HCHK(hipMemsetAsync(S_->delta, 0, (size_t)std::max<int64_t>(n, 1) * sizeof(double), s_));
    if (n == 0) return;
    HCHK(hipMemcpyAsync(S_->ctl, S_->ctl0, sizeof(mvba::CgCtl), hipMemcpyDeviceToDevice, s_));
    if (pq_atomic()) HCHK(hipMemsetAsync(S_->scal + kPqSlot, 0, 2 * sizeof(double), s_));
    // b.b straight into the control block: the first update's finalisation stops
    // the solve at |b| = 0 (Ceres: "Convergence. |b| = 0.", x = 0), so the host
    // does not wait for it (one stream sync per linear solve less)
    HCHK(mvba_launch_dot(n, S_->b, S_->b, S_->partial, S_->cnt + 6, &S_->ctl->bb, s_));
    const mvba::FrameDirZ fz{h_->d_frame_lin, h_->d_fd, h_->d_frec, S_->dirz, (int32_t)h_->nframes, 0};
    HCHK(mvba_launch_cg_update(n, S_->ent, S_->fac, 4 | 8, 0.0, S_->p, nullptr, S_->b, S_->delta, S_->r, S_->r2,
                               S_->z, S_->partial, S_->cnt, S_->scal + 8, S_->ctl, mvba::kIterFromCtl,
                               fused_dir() && !dz_in_pass_a() ? &fz : nullptr, nullptr, nullptr, s_));
  }

  // The template control block of this solve's linear solves (options only)
  void upload_ctl0() {
    mvba::CgCtl c{};
    c.eta = o_.eta;
    c.min_iter = o_.min_linear_solver_iterations;
    c.max_iter = o_.max_linear_solver_iterations;
    c.it = 0;
    *S_->hctl = c;
    HCHK(hipMemcpyAsync(S_->ctl0, S_->hctl, sizeof(mvba::CgCtl), hipMemcpyHostToDevice, s_));
    HCHK(hipStreamSynchronize(s_));  // hctl[0] is reused for the solves' results
  }

  // Everything a step computes before its CG iterations, enqueue only: LM
  // damping (1/radius from scal[kRadSlot]), block-Jacobi preconditioner, Schur
  // right-hand side, CG start. One captured graph per handle when graphs are on.
  void step_prologue(double radius) {
    S_->hscal[kRadSlot] = 1.0 / radius;  // the previous step's copy completed (its fetch synchronised)
    HCHK(hipMemcpyAsync(S_->scal + kRadSlot, S_->hscal + kRadSlot, sizeof(double), hipMemcpyHostToDevice, s_));
    // the per-slot records (landmark + Cauchy weight sqrt(rho')) were written
    // by K2 at this linearization point (h_->lin_obsx). A landmark-only copy
    // would carry the prep kernel's free flag in .w, which the frame-order
    // passes would take as the Cauchy weight: never fall back to one.
    if (obsx() && h_->lin_obsx != obsx())
      throw StatusErr{MVBA_E_INVALID, "internal: CG slot records were not written by the linearization"};
    refresh_graph_sig();
    enqueue_seq(0, [&] {
      HCHK(mvba_launch_lm_diag(S_->nc, S_->cdiag, o_.jacobi_scaling ? S_->sc : nullptr, 0.0, S_->scal + kRadSlot,
                               o_.min_lm_diagonal, o_.max_lm_diagonal, S_->dmp, s_));
      HCHK(mvba_launch_block_prec(S_->nblocks, S_->max_bsize, S_->goff, S_->hoff, S_->bsize, S_->lin + S_->ng,
                                  S_->dmp, S_->fac, s_));
      schur_rhs();
      cg_start();
    });
  }
  static constexpr int kRadSlot = 20;  // scal[20]: 1/radius of the current step

  // PCG on S delta_c = b (conjugate_gradients_solver.cc [ext]) with every
  // scalar step on the device (CgCtl): iterations are enqueued in batches and
  // gated by ctl->done, one host read per batch. Sharded solves run the same
  // loop: the per-iteration exchange of the product is stream-ordered and the
  // replicated camera-side state gives every rank the same stopping decisions.
  // The start (cg_start) is part of the step prologue.
  //
  // Every launch argument of iteration i is a function of i mod 10 (the
  // double-buffered p, r, direction records and p.q accumulator by the parity
  // of i, the residual reset at i % 10 == 0; the iteration number itself is
  // counted on the device, CgCtl::it), so solves capture runs of iterations as
  // hipGraphs once per handle and replay them (RCCL-sharded solves too, with
  // the exchange inside the graph): a batch of k iterations costs a few graph
  // launches instead of 5 k kernel launches, whose host time (≈ 25 us per
  // iteration, 5-6 us per hipLaunchKernel) bound the CG iteration of small
  // problems (profiles/r05/r05b/s8_timing_r05b.log: enqueue 27.6 us vs 16.1 us
  // of wait per iteration on the 1/8 c2 shard).
  CgResult cg_device() {
    CgResult R;
    const int64_t n = S_->ng;
    double* xv = S_->delta;
    if (n == 0) return R;
    const int32_t* gate = &S_->ctl->done;
    const bool fused_dir = this->fused_dir();
    const bool dz_pa = dz_in_pass_a();
    const mvba::FrameDirZ fz{h_->d_frame_lin, h_->d_fd, h_->d_frec, S_->dirz, (int32_t)h_->nframes, 0};
    // p[i & 1] = the direction of iteration i (p[(i - 1) & 1] the previous
    // one), r[i & 1] = the residual iteration i starts from, dirp likewise
    double* const P[2] = {S_->p, S_->p2};
    double* const Rv[2] = {S_->r, S_->r2};
    // The host learns where a batch ended from the CgMirror its last update
    // launch writes into host-coherent memory (one spin on a pinned word), not
    // from a device-to-host copy launch and an event after it. Every run of
    // iterations (graph) or eager batch ends with one such launch; the host
    // counts them. MVBA_CG_MIRROR=0 (read per call): the copy and the event.
    // Pipelined batches keep the copies (two batches in flight).
    const char* pipe_env = std::getenv("MVBA_CG_PIPE");  // read per call
    const bool pipelined = pipe_env && pipe_env[0] == '1';
    const bool mirror = mirror_on();
    mvba::CgMirror* const mir = mirror ? S_->dmir : nullptr;
    uint32_t mir_expected = 0;
    if (mirror) __atomic_store_n(&S_->hmir->seq, 0u, __ATOMIC_RELEASE);  // ctl->mseq restarts with cg_start
    auto upd = [&](int32_t mode, const double* q, const double* p, const double* r_in, double* r_out,
                   mvba::CgMirror* m = nullptr) {
      HCHK(mvba_launch_cg_update(n, S_->ent, S_->fac, mode, 0.0, p, q, S_->b, xv, r_in, r_out, S_->z, S_->partial,
                                 S_->cnt, S_->scal + 8, S_->ctl, mvba::kIterFromCtl,
                                 fused_dir && !dz_pa ? &fz : nullptr, (mode & 1) && q ? pq_of(q) : nullptr, m, s_));
    };
    const int imax = std::max(o_.max_linear_solver_iterations, 1);
    // the fused CG step: iteration i's pass A carries the update of iteration
    // i - 1 (deferred by body(i - 1)), except at the start of a run of
    // iterations (a graph run or an eager batch ends with its update, so the
    // host's control-block read sees it) and after a residual reset
    const bool fuse = fused_step();
    const double* pending_pq = nullptr;  // the deferred update's p.q (its iteration's parity)
    bool pending = false;
    const Group& G0 = h_->groups[0];
    const bool chunked = pass_a_chunked();
    const bool co_slot = co_slot_order(std::getenv("MVBA_CO_ORDER"));
    auto body = [&](int i, bool run_end) {
      const mvba::LazyDir lz{S_->z, P[(i - 1) & 1], P[i & 1], n, S_->ctl, 0, 0.0};
      cg_par_ = i & 1;
      if (pending) {
        // update of iteration i - 1 (mode 1|2|8) + pass A of iteration i
        HCHK(mvba_launch_upd_pass_a(G0.model, G0.deg, n, S_->ent, S_->fac, P[(i - 1) & 1], S_->q, S_->b, xv,
                                    Rv[(i - 1) & 1], Rv[i & 1], S_->z, S_->partial, S_->cnt, S_->scal + 8, S_->ctl,
                                    pending_pq, chunked ? h_->d_achunks + G0.achunk_begin
                                                        : h_->d_segchunks + G0.seg_begin,
                                    chunked ? G0.achunk_count : G0.seg_count, h_->d_frame_lin, h_->d_fd, h_->d_frec,
                                    S_->dirp[(i - 1) & 1], S_->dirz, co_slot ? nullptr : h_->d_slot_po,
                                    (double4*)S_->cbuf, S_->cbuf2, S_->prec, obsx(), s_));
        // w_p from c_z + beta c_p; its frame blocks form this iteration's
        // direction records d = d_z + beta d_p
        mvba::FusedStep fs;
        fs.dz = S_->dirz;
        fs.dp = S_->dirp[(i - 1) & 1];
        fs.dp_out = S_->dirp[i & 1];
        fs.fd = h_->d_fd;
        fs.fl = h_->d_frame_lin;
        fs.ctl = S_->ctl;
        fs.cbuf2 = S_->cbuf2;
        fs.nframes = (int32_t)h_->nframes;
        HCHK(mvba_launch_point_w(h_->npts, h_->d_pt_begin, co_slot ? h_->d_po_slot : nullptr,
                                 (const double4*)S_->cbuf, nullptr, S_->phess, S_->dmp + S_->ng, h_->d_pts, S_->wbuf,
                                 4, gate, nullptr, nullptr, &fs, s_));
        reduce_frames(S_->q, lz.p_new, 0, S_->dirp[i & 1], gate, S_->ctl, &lz);
        pending = false;
      } else if (fused_dir) {
        apply_schur_cg(S_->q, gate, S_->ctl, lz,
                       mvba::DirPair{dz_pa ? nullptr : S_->dirz, S_->dirp[(i - 1) & 1], S_->dirp[i & 1], S_->ctl,
                                     lz.z, lz.p_old, h_->d_frame_lin, dz_pa ? h_->d_frec : nullptr});
      } else {
        apply_schur(P[i & 1], S_->q, 0, gate, S_->ctl, &lz);
      }
      double* r_in = Rv[i & 1];
      double* r_out = Rv[(i + 1) & 1];
      if (i % 10 == 0) {  // residual reset: r = b - A x
        upd(1, S_->q, P[i & 1], r_in, nullptr);
        apply_schur(xv, S_->tmp, 1, gate, nullptr);
        upd(4 | 8, S_->tmp, P[i & 1], r_in, r_out, run_end ? mir : nullptr);
      } else if (fuse && !run_end && i < imax) {
        pending = true;  // into the next iteration's pass A
        pending_pq = pq_of(S_->q);
      } else {
        upd(1 | 2 | 8, S_->q, P[i & 1], r_in, r_out, run_end ? mir : nullptr);
      }
    };
    refresh_graph_sig();
    const bool use_graphs = graphs_enabled();
    // iterations [i, i + L) with i's offset o = (i - 1) % 10 and L <= 10 - o:
    // one replay of the captured run (captured on first use)
    auto run_chunk = [&](int i, int L) {
      const int o = (i - 1) % 10;
      for (const SolverState::CgGraph& g : S_->graphs)
        if (g.o == o && g.L == L) {
          HCHK(hipGraphLaunch(g.exec, s_));
          graph_launches_++;
          return;
        }
      hipGraphExec_t exec = nullptr;
      if (!capture([&] {
            for (int k = 0; k < L; k++) body(i + k, k == L - 1);
          }, &exec)) {
        pending = false;  // the failed capture's deferred update never ran: the run again, eagerly
        for (int k = 0; k < L; k++) body(i + k, k == L - 1);  // this run eagerly; later ones too
        return;
      }
      S_->graphs.push_back(SolverState::CgGraph{o, L, exec});
      HCHK(hipGraphLaunch(exec, s_));
      graph_launches_++;
    };
    int i = 1;
    // Batch sizes only decide where the host looks at the control block (gated
    // iterations past the stop are no-ops): the first batch runs to just short
    // of the previous solve's iteration count, later ones are short, so most
    // solves need one or two host reads and few gated iterations.
    // The second batch is 2 (the previous count is the usual ending), then 4;
    // MVBA_CG_BATCH2 sets the second (A/B timing). A gated iteration costs
    // ≈ 20 us at c2 and ≈ 36 us at c3 (a gated pass B alone is 10 us there).
    static const int second = std::getenv("MVBA_CG_BATCH2") ? std::max(1, std::atoi(std::getenv("MVBA_CG_BATCH2"))) : 2;
    int first = std::max(4, last_cg_iters_ - 2);
    // graph run length: 10 (one run per reset period) for long solves, shorter
    // runs (aligned to the period: 5, 2, 1) when the previous solve was short,
    // so rounding a batch up to whole runs adds few gated iterations (a gated
    // iteration still dispatches every block of its five launches: ~36 us at
    // c3, whose solves take 3-8 CG iterations; profiles/r05/r05h/).
    // MVBA_CG_GRAPH_RUN fixes it (A/B timing).
    const int kGraphRun = [&] {
      if (const char* e = std::getenv("MVBA_CG_GRAPH_RUN")) return std::max(1, std::min(10, std::atoi(e)));
      const int last = std::max(last_cg_iters_, 1);
      return last >= 40 ? 10 : last >= 10 ? 5 : last >= 4 ? 2 : 1;
    }();
    if (use_graphs) first = (first + kGraphRun - 1) / kGraphRun * kGraphRun;
    // Pipelined batches (MVBA_CG_PIPE=1, read per call): the next batch is
    // enqueued before the host waits for the previous one's control block (a
    // pinned copy per batch, read after its event), so the GPU does not idle
    // through the host's turnaround, but a stop seen in batch k leaves batch
    // k + 1 to run as gated no-ops ahead of the back-substitution. Same box
    // (profiles/r05/r05k/): CG loop 42.5 vs 42.2 us per iteration (1/8 c2
    // shard), 73.6 vs 74.0 (c2), back-substitution +46 / +64 us per solve
    // behind the gated batch: not the default.
    auto enqueue_batch = [&](int batch, int slot) {
      if (use_graphs) batch = (batch + kGraphRun - 1) / kGraphRun * kGraphRun;
      const double tb0 = now_s();
      if (cg_timing()) tm_.batches++;
      const int iend = std::min(i + batch, imax + 1);  // iterations [i, iend)
      if (cg_timing()) tm_.enqueued += iend - i;
      if (use_graphs && !S_->graphs_broken) {
        // runs of kGraphRun iterations aligned to the reset period (10: one run
        // per period, captured by the first solve that reaches iteration 10;
        // batches round up to whole runs); a shorter tail only at
        // max_linear_solver_iterations. Same-box A/B (profiles/r05/r05d/): the
        // 1/8 c2 shard's CG loop 43.5-44.0 us per iteration eager, 42.7 with
        // runs of 2, 40.8-41.1 with runs of 10; c2 76.7-77.1 / 79.6 / 76.6-76.9
        // (GPU-bound there: the graph removes host time, not GPU-side gaps)
        while (i < iend) {
          const int o = (i - 1) % 10;
          const int L = std::min({kGraphRun - o % kGraphRun, 10 - o, imax + 1 - i});
          run_chunk(i, L);
          i += L;
          mir_expected++;  // the run's last update mirrors
        }
      } else {
        for (; i < iend; i++) body(i, i == iend - 1);
        mir_expected++;
      }
      if (!mirror) {
        HCHK(hipMemcpyAsync(S_->hctl + slot, S_->ctl, sizeof(mvba::CgCtl), hipMemcpyDeviceToHost, s_));
        HCHK(hipEventRecord(S_->ev_cg[slot - 1], s_));
      }
      if (cg_timing()) tm_.enqueue += now_s() - tb0;
    };
    auto wait_batch = [&](int slot) -> const mvba::CgCtl& {
      const double tw = now_s();
      if (mirror) {
        // spin on the pinned seq word; every 4096 polls ask the stream, so a
        // failed launch (which never writes the mirror) surfaces as its error
        const uint32_t want = mir_expected;
        for (unsigned k = 1; __atomic_load_n(&S_->hmir->seq, __ATOMIC_ACQUIRE) != want; k++) {
          if (k % 4096 == 0) {
            const hipError_t e = hipStreamQuery(s_);
            if (e == hipSuccess && __atomic_load_n(&S_->hmir->seq, __ATOMIC_ACQUIRE) != want)
              throw StatusErr{MVBA_E_INVALID, "internal: CG batch ended without its control mirror"};
            if (e != hipSuccess && e != hipErrorNotReady) HCHK(e);
          }
          __builtin_ia32_pause();
        }
        mvba::CgCtl& c = S_->hctl[slot];
        c.done = S_->hmir->done;
        c.status = S_->hmir->status;
        c.iters = S_->hmir->iters;
      } else {
        HCHK(hipEventSynchronize(S_->ev_cg[slot - 1]));
      }
      if (cg_timing()) tm_.wait += now_s() - tw;
      return S_->hctl[slot];
    };
    int slot = 1;
    enqueue_batch(first, slot);
    const mvba::CgCtl* last = nullptr;
    for (int nb = 0;;) {
      const int next = 3 - slot;
      bool ahead = false;
      if (pipelined && i <= imax) {
        enqueue_batch((++nb == 1) ? second : 4, next);
        ahead = true;
      }
      last = &wait_batch(slot);
      if (last->done) break;
      if (i > imax) {  // every iteration is enqueued: the newest batch's state is final (stopped at max_iter)
        if (ahead) last = &wait_batch(next);
        break;
      }
      if (!ahead) enqueue_batch((++nb == 1) ? second : 4, next);
      slot = next;
    }
    *S_->hctl = *last;
    R.iters = S_->hctl->iters;
    R.status = S_->hctl->status;
    last_cg_iters_ = R.iters;
    return R;
  }

  // delta_p = -(V+D)^-1 (g_p + W' delta_c); returns model cost change -(g'delta + |J delta|^2 / 2)
  // (fetch_now false: enqueue only, the three terms land in scal[0..2]). The
  // enqueues are one captured graph per handle when graphs are on.
  double back_substitute(bool fetch_now = true) {
    enqueue_seq(1, [&] { back_substitute_enqueue(); });
    if (!fetch_now) return 0.0;
    return model_change(fetch(3));
  }
  void back_substitute_enqueue() {
    HCHK(mvba_launch_frame_dir(h_->d_frame_lin, (int32_t)h_->nframes, h_->d_fd, h_->d_frec, S_->delta, S_->dir,
                               nullptr, nullptr, s_));
    // |J delta|^2 over the local reprojection and depth blocks -> scal[0].
    // Reprojection-only problems with one model group: frame-order pass A +
    // k_point_w (w_p into delta_p) + the |u_o|^2 sweep k_pass_sq; otherwise
    // (depth blocks, XYZ priors, several models) the point-order pass, whose
    // per-observation gathers of frame records outgrow the L2 at c3. Kernel
    // traces (profiles/r03/ab_backsub/): c3 514 vs 760 us, c2 57 vs 59 us per
    // solve. MVBA_BACKSUB=point forces the point-order pass, for A/B timing.
    const char* bs_env = std::getenv("MVBA_BACKSUB");  // read per call: tests switch it
    const bool frame_order = !(bs_env && !std::strcmp(bs_env, "point")) && h_->ndep == 0 && h_->nxyz == 0 &&
                             h_->groups.size() == 1 && h_->groups[0].seg_count > 0 && obsx();
    if (frame_order) {
      const Group& G = h_->groups[0];
      const char* co_env = std::getenv("MVBA_CO_ORDER");  // read per call: tests switch it
      const bool co_slot = co_slot_order(co_env);
      HCHK(mvba_launch_pass_a_frame(G.model, G.deg, h_->d_segchunks + G.seg_begin, G.seg_count, h_->d_segs,
                                    h_->d_pts, h_->d_obs_pid, h_->d_obs_meas, co_slot ? nullptr : h_->d_slot_po,
                                    plain_dir(S_->dir), (double4*)S_->cbuf, flags_, cauchy_c_, nullptr, S_->prec,
                                    obsx(), s_));
      if (point_w_tiles())
        HCHK(mvba_launch_point_w_seg(h_->nwtiles, h_->d_wtiles, h_->d_wlane_pid,
                                     co_slot ? h_->d_wlane_slot : h_->d_wlane_pos, h_->d_pt_begin,
                                     co_slot ? h_->d_po_slot : nullptr, (const double4*)S_->cbuf, S_->G + S_->ng,
                                     S_->phess, S_->dmp + S_->ng, h_->d_pts, S_->delta + S_->ng, 3, nullptr, s_));
      else
        HCHK(mvba_launch_point_w(h_->npts, h_->d_pt_begin, co_slot ? h_->d_po_slot : nullptr,
                                 (const double4*)S_->cbuf, S_->G + S_->ng, S_->phess, S_->dmp + S_->ng, h_->d_pts,
                                 S_->delta + S_->ng, 3, nullptr, nullptr, nullptr, nullptr, s_));
      HCHK(mvba_launch_pass_sq(G.model, G.deg, h_->d_segchunks + G.seg_begin, G.seg_count, h_->d_obs_pid,
                               plain_dir(S_->dir), S_->delta + S_->ng, 3, S_->prec, obsx(), S_->partial,
                               S_->cnt + 5, S_->scal + 0, s_));
    } else {
      HCHK(mvba_launch_pass_a(pa_model(), pa_deg(), h_->d_pt_begin, h_->npts, h_->d_po_frame, h_->d_po_meas,
                              h_->d_fd, h_->d_frec, h_->d_params, h_->d_pts, S_->dir, S_->G + S_->ng, S_->phess,
                              S_->dmp + S_->ng, S_->zbuf, S_->delta + S_->ng, 3, S_->partial, S_->cnt + 5,
                              S_->scal + 0, flags_, cauchy_c_, h_->point_extra(), S_->delta, S_->du, nullptr,
                              S_->prec, s_));
    }
    HCHK(mvba_launch_axpby(3 * S_->np, -1.0, S_->delta + S_->ng, 0.0, nullptr, S_->delta + S_->ng, s_));
    dot(3 * S_->np, S_->G + S_->ng, S_->delta + S_->ng, 1);  // g_p' delta_p (local points)
    exchange(S_->scal, 2, MVBA_REDUCE_SUM);
    dot(S_->ng, S_->G, S_->delta, 2);  // g_c' delta_c (global already)
  }
  // the model cost change from the back-substitution's scal[0..2]
  double model_change(const double* hs) {
    for (int k = 0; k < 3; k++) last_mc_[k] = hs[k];
    return -(hs[1] + hs[2] + 0.5 * hs[0]);
  }
  double last_mc_[3] = {0, 0, 0};  // |J delta|^2, g_p'delta_p, g_c'delta_c of the last step

  // max |x - P(x - g)| and |x - P(x - g)|, over ranks
  double grad_max_norm() {
    // camera part is identical on every rank: take it from the compact vector once,
    // points part is rank-local; MAX-reduce the combination.
    HCHK(mvba_launch_proj_grad_max(S_->nc, S_->x, S_->G, S_->lo, S_->hi, S_->partial, S_->scal + 0, s_));
    exchange(S_->scal, 1, MVBA_REDUCE_MAX);
    return fetch(1)[0];
  }

  // |x|^2 split: camera part (global) + point part summed over ranks
  double norm2_compact(const double* v) {
    dot(3 * S_->np, v + S_->ng, v + S_->ng, 0);
    exchange(S_->scal, 1, MVBA_REDUCE_SUM);
    dot(S_->ng, v, v, 1);
    const double* hs = fetch(2);
    return hs[0] + hs[1];
  }

  double step_norm2() {  // |xn - x|^2, difference formed explicitly
    HCHK(mvba_launch_axpby(S_->nc, 1.0, S_->xn, -1.0, S_->x, S_->scr, s_));
    return norm2_compact(S_->scr);
  }

  // a.b over the compact vector: camera part is replicated on every rank, point part summed
  double dot_global(const double* a, const double* b) {
    dot(3 * S_->np, a + S_->ng, b + S_->ng, 0);
    exchange(S_->scal, 1, MVBA_REDUCE_SUM);
    dot(S_->ng, a, b, 1);
    const double* hs = fetch(2);
    return hs[0] + hs[1];
  }

  void set_params_from(const double* v) {
    HCHK(mvba_launch_scatter(S_->ng, S_->cam_poff, S_->np, h_->d_pt_off, h_->d_pt_free, v, h_->d_params, s_));
  }

  double armijo(double x_cost, double gtd, bool* relinearized);
};

// ---- polynomial interpolation of the line search (Ceres polynomial.cc [ext])
struct Sample {
  double x = 0.0, f = 0.0, g = 0.0;
  bool fv = false, gv = false;
};

double poly_eval(const std::vector<double>& c, double x) {  // highest degree first
  double v = 0.0;
  for (double a : c) v = v * x + a;
  return v;
}

// FindInterpolatingPolynomial: value and gradient constraints, square system.
std::vector<double> interpolating_polynomial(const std::vector<Sample>& smp) {
  int m = 0;
  for (const Sample& s : smp) m += (s.fv ? 1 : 0) + (s.gv ? 1 : 0);
  const int deg = m - 1;
  std::vector<double> A((size_t)m * m, 0.0), rhs(m, 0.0);
  int row = 0;
  for (const Sample& s : smp) {
    if (s.fv) {
      for (int j = 0; j <= deg; j++) A[row * m + j] = std::pow(s.x, deg - j);
      rhs[row++] = s.f;
    }
    if (s.gv) {
      for (int j = 0; j < deg; j++) A[row * m + j] = (deg - j) * std::pow(s.x, deg - j - 1);
      rhs[row++] = s.g;
    }
  }
  // Gaussian elimination with partial pivoting (m <= 6)
  std::vector<int> perm(m);
  for (int i = 0; i < m; i++) perm[i] = i;
  for (int k = 0; k < m; k++) {
    int piv = k;
    for (int i = k + 1; i < m; i++)
      if (std::fabs(A[i * m + k]) > std::fabs(A[piv * m + k])) piv = i;
    if (piv != k) {
      for (int j = 0; j < m; j++) std::swap(A[k * m + j], A[piv * m + j]);
      std::swap(rhs[k], rhs[piv]);
    }
    const double d = A[k * m + k];
    if (d == 0.0) continue;
    for (int i = k + 1; i < m; i++) {
      const double f = A[i * m + k] / d;
      for (int j = k; j < m; j++) A[i * m + j] -= f * A[k * m + j];
      rhs[i] -= f * rhs[k];
    }
  }
  std::vector<double> c(m, 0.0);
  for (int i = m - 1; i >= 0; i--) {
    double v = rhs[i];
    for (int j = i + 1; j < m; j++) v -= A[i * m + j] * c[j];
    c[i] = (A[i * m + i] != 0.0) ? v / A[i * m + i] : 0.0;
  }
  return c;
}

// Real parts of all roots (FindPolynomialRoots with imaginary == NULL), Durand-Kerner.
std::vector<double> root_real_parts(std::vector<double> c) {
  while (!c.empty() && c[0] == 0.0) c.erase(c.begin());
  const int n = (int)c.size() - 1;
  std::vector<double> out;
  if (n < 1) return out;
  if (n == 1) {
    out.push_back(-c[1] / c[0]);
    return out;
  }
  if (n == 2) {
    const double a = c[0], b = c[1], cc = c[2], disc = b * b - 4 * a * cc;
    if (disc < 0) {
      out.push_back(-b / (2 * a));
      out.push_back(-b / (2 * a));
    } else {
      const double sq = std::sqrt(disc);
      out.push_back((-b + sq) / (2 * a));
      out.push_back((-b - sq) / (2 * a));
    }
    return out;
  }
  typedef std::complex<double> cd;
  std::vector<cd> z(n);
  const cd seed(0.4, 0.9);
  z[0] = 1.0;
  for (int i = 1; i < n; i++) z[i] = z[i - 1] * seed;
  auto P = [&](cd x) {
    cd v = 0.0;
    for (double a : c) v = v * x + a / c[0];
    return v;
  };
  for (int it = 0; it < 500; it++) {
    double moved = 0.0;
    for (int i = 0; i < n; i++) {
      cd den = 1.0;
      for (int j = 0; j < n; j++)
        if (j != i) den *= (z[i] - z[j]);
      const cd dz = P(z[i]) / den;
      z[i] -= dz;
      moved = std::max(moved, std::abs(dz));
    }
    if (moved < 1e-15) break;
  }
  for (const cd& r : z) out.push_back(r.real());
  return out;
}

// MinimizeInterpolatingPolynomial over [lo, hi]
double minimize_interpolant(const std::vector<Sample>& smp, double lo, double hi) {
  const std::vector<double> poly = interpolating_polynomial(smp);
  double bx = 0.5 * (lo + hi), bv = poly_eval(poly, bx);
  auto consider = [&](double x) {
    if (x < lo || x > hi) return;
    const double v = poly_eval(poly, x);
    if (v < bv) {
      bv = v;
      bx = x;
    }
  };
  consider(lo);
  consider(hi);
  if (poly.size() > 2) {
    std::vector<double> der;
    const int deg = (int)poly.size() - 1;
    for (int j = 0; j < deg; j++) der.push_back(poly[j] * (deg - j));
    for (double r : root_real_parts(der)) consider(r);
  }
  for (const Sample& s : smp) consider(s.x);
  return bx;
}

// Projected Armijo search along delta (TrustRegionMinimizer::DoLineSearch with
// ARMIJO + CUBIC interpolation [ext]): scales delta in place on success.
double Solver::armijo(double x_cost, double gtd, bool* relinearized) {
  const double kSuff = 1e-4, kMaxContr = 1e-3, kMinContr = 0.6, kMinStep = 1e-9;
  const int kMaxIter = 20;
  HCHK(mvba_launch_proj_grad_max(S_->nc, S_->delta, S_->delta, nullptr, nullptr, S_->partial, S_->scal, s_));
  exchange(S_->scal, 1, MVBA_REDUCE_MAX);
  const double dmax = fetch(1)[0];
  auto eval = [&](double a, bool want_grad) {
    Sample smp;
    smp.x = a;
    HCHK(mvba_launch_axpby(S_->nc, a, S_->delta, 0.0, nullptr, S_->scr, s_));
    HCHK(mvba_launch_plus(S_->nc, S_->x, S_->scr, S_->lo, S_->hi, S_->xn, s_));
    set_params_from(S_->xn);
    smp.f = cost();
    smp.fv = std::isfinite(smp.f);
    if (want_grad && smp.fv) {
      linearize();
      *relinearized = true;
      smp.g = dot_global(S_->delta, S_->G);
      smp.gv = std::isfinite(smp.g);
    }
    return smp;
  };
  Sample init;
  init.x = 0.0;
  init.f = x_cost;
  init.g = gtd;
  init.fv = init.gv = true;
  Sample prev, cur = eval(1.0, false);
  int it = 0;
  while (!cur.fv || cur.f > x_cost + kSuff * gtd * cur.x) {
    if (++it >= kMaxIter) return 1.0;
    double step;
    if (!cur.fv) {
      step = std::min(std::max(cur.x * 0.5, kMaxContr * cur.x), kMinContr * cur.x);
    } else {
      if (!cur.gv) cur = eval(cur.x, true);
      std::vector<Sample> smp{init, cur};
      if (prev.fv) smp.push_back(prev);
      step = minimize_interpolant(smp, kMaxContr * cur.x, kMinContr * cur.x);
    }
    if (step * dmax < kMinStep) return 1.0;
    prev = cur;
    cur = eval(step, false);
  }
  if (cur.x != 1.0) HCHK(mvba_launch_axpby(S_->nc, cur.x, S_->delta, 0.0, nullptr, S_->delta, s_));
  return cur.x;
}

void Solver::run(mvba_solver_summary* sum) {
  const double t0 = now_s();
  const int64_t nc = S_->nc;
  // bounds in compact form (+-inf for constant points)
  bounded_ = false;
  if (S_->lo) (void)hipFree(S_->lo);
  if (S_->hi) (void)hipFree(S_->hi);
  S_->lo = S_->hi = nullptr;
  if (o_.lower_bounds || o_.upper_bounds) {
    std::vector<int64_t> pt_off(S_->np);
    std::vector<uint8_t> pt_free(S_->np);
    if (S_->np) {
      HCHK(hipMemcpy(pt_off.data(), h_->d_pt_off, S_->np * sizeof(int64_t), hipMemcpyDeviceToHost));
      HCHK(hipMemcpy(pt_free.data(), h_->d_pt_free, S_->np, hipMemcpyDeviceToHost));
    }
    const double inf = std::numeric_limits<double>::infinity();
    auto build = [&](const double* src, double fill, double** dst) {
      if (!src) return;
      std::vector<double> v(nc, fill);
      for (int64_t e = 0; e < S_->ng; e++) v[e] = src[h_->cam_poff[e]];
      for (int64_t p = 0; p < S_->np; p++)
        if (pt_free[p])
          for (int c = 0; c < 3; c++) v[S_->ng + 3 * p + c] = src[pt_off[p] + c];
      for (double b : v)
        if (std::isfinite(b)) bounded_ = true;
      HCHK(upload(dst, v));
    };
    build(o_.lower_bounds, -inf, &S_->lo);
    build(o_.upper_bounds, inf, &S_->hi);
  }

  // Nothing to optimize (no residual blocks, or every block constant): Ceres
  // 1.14 returns CONVERGENCE with the cost evaluated once (solver.cc [ext]).
  {
    double nfree = (double)S_->ng;
    if (nfree == 0.0 && S_->np > 0) {
      std::vector<uint8_t> pt_free(S_->np);
      HCHK(hipMemcpy(pt_free.data(), h_->d_pt_free, S_->np, hipMemcpyDeviceToHost));
      for (uint8_t f : pt_free) nfree += f ? 1.0 : 0.0;
    }
    if (o_.allreduce) {
      HCHK(hipMemcpyAsync(S_->scal, &nfree, sizeof(double), hipMemcpyHostToDevice, s_));
      exchange(S_->scal, 1, MVBA_REDUCE_MAX);
      nfree = fetch(1)[0];
    }
    if (nfree == 0.0) {
      const double c = cost();
      sum->initial_cost = sum->final_cost = c;
      sum->num_successful_steps = 0;
      sum->termination_type = MVBA_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message),
                    "Function tolerance reached. No non-constant parameter blocks found.");
      sum->total_time_s = now_s() - t0;
      return;
    }
  }
  HCHK(mvba_launch_gather(S_->ng, S_->cam_poff, S_->np, h_->d_pt_off, h_->d_pt_free, h_->d_params, S_->x, s_));
  upload_ctl0();
  double tl = now_s();
  double x_cost = linearize();
  sum->linearize_time_s += now_s() - tl;
  sum->initial_cost = x_cost;
  if (o_.jacobi_scaling) HCHK(mvba_launch_jacobi_scale(nc, S_->cdiag, S_->sc, s_));
  double gmax = grad_max_norm();
  double x_norm = std::sqrt(norm2_compact(S_->x));
  double radius = o_.initial_trust_region_radius, decrease = 2.0;
  int iteration = 0, invalid = 0;
  bool successful = true;
  sum->num_successful_steps = 1;  // iteration 0 counts, as in Ceres' summary
  auto row = [&](double cost, double change, double step, double ratio, int ls, double it_time) {
    if (!o_.progress_to_stdout) return;
    if (iteration == 0)
      std::printf("iter      cost      cost_change  |gradient|   |step|    tr_ratio  tr_radius  ls_iter  "
                  "iter_time  total_time\n");
    std::printf("% 4d % 8e   % 3.2e   % 3.2e  % 3.2e  % 3.2e % 3.2e     % 4d   % 3.2e   % 3.2e\n", iteration, cost,
                change, gmax, step, ratio, radius, ls, it_time, now_s() - t0);
    std::fflush(stdout);
  };
  row(x_cost, 0.0, 0.0, 0.0, 0, now_s() - t0);
  auto finish = [&](int type, const std::string& msg) {
    sum->termination_type = type;
    std::snprintf(sum->message, sizeof(sum->message), "%s", msg.c_str());
  };
  char buf[256];
  for (;;) {
    // FinalizeIterationAndCheckIfMinimizerCanContinue
    if (iteration >= o_.max_num_iterations) {
      std::snprintf(buf, sizeof(buf), "Maximum number of iterations reached. Number of iterations: %d.", iteration);
      finish(MVBA_NO_CONVERGENCE, buf);
      break;
    }
    if (successful && gmax <= o_.gradient_tolerance) {
      std::snprintf(buf, sizeof(buf), "Gradient tolerance reached. Gradient max norm: %e <= %e", gmax,
                    o_.gradient_tolerance);
      finish(MVBA_CONVERGENCE, buf);
      break;
    }
    if (radius <= o_.min_trust_region_radius) {
      std::snprintf(buf, sizeof(buf), "Minimum trust region radius reached. Trust region radius: %e <= %e", radius,
                    o_.min_trust_region_radius);
      finish(MVBA_CONVERGENCE, buf);
      break;
    }
    iteration++;
    const double it0 = now_s();
    // ComputeTrustRegionStep (LevenbergMarquardtStrategy::ComputeStep)
    const double ts = now_s();
    step_prologue(radius);  // damping, preconditioner, right-hand side, CG start
    if (cg_timing()) {
      HCHK(hipStreamSynchronize(s_));
      tm_.rhs += now_s() - ts;
      tm_.solves++;
    }
    const CgResult cgr = cg_device();
    sum->num_linear_iterations += cgr.iters;
    if (cg_timing()) tm_.iters += cgr.iters;
    bool valid = cgr.status != 2;
    double mcc = 0.0;
    // Merged step (unbounded problems; MVBA_LM_MERGED=0: one host read per
    // quantity, as before): the candidate x + delta, its cost and |step| are
    // enqueued behind the back-substitution and read back together with the
    // model cost change and the device error word, one stream sync instead of
    // four. An invalid step then restores the parameters it moved.
    const bool merged = !bounded_ && merged_reads();
    double m_cand = 0.0, m_step2 = 0.0, m_eval_gpu_s = 0.0;
    // test hook (read per call): the first N steps of the solve are declared
    // invalid after their model change is known, as a non-positive or NaN model
    // change would be (both read paths must then end the same way)
    const char* fi_env = std::getenv("MVBA_TEST_INVALID_STEPS");
    const bool forced_invalid = fi_env && iteration <= std::atoi(fi_env);
    if (valid) {
      const double tbs = now_s();
      mvba_status cand_err = MVBA_OK;
      if (merged) {
        back_substitute(false);
        HCHK(hipEventRecord(S_->ev[0], s_));
        HCHK(mvba_launch_plus(nc, S_->x, S_->delta, S_->lo, S_->hi, S_->xn, s_));
        set_params_from(S_->xn);
        cost_enqueue();
        HCHK(mvba_launch_axpby(S_->nc, 1.0, S_->xn, -1.0, S_->x, S_->scr, s_));
        norm2_enqueue(S_->scr, 3, 4);
        HCHK(hipEventRecord(S_->ev[1], s_));
        // the candidate's device error (K0's alpha range check,
        // rig_calibrator.cc:346) is raised only for a valid step: Ceres rejects
        // an invalid step without evaluating its candidate
        const double* hs = fetch_checked(17, &cand_err);
        mcc = model_change(hs);
        m_cand = hs[16];
        m_step2 = hs[3] + hs[4];
        float ms = 0.0f;
        HCHK(hipEventElapsedTime(&ms, S_->ev[0], S_->ev[1]));
        m_eval_gpu_s = 1e-3 * ms;  // the candidate's share of the wait (eval time)
      } else {
        mcc = back_substitute();
      }
      if (cg_timing()) tm_.backsub += now_s() - tbs - m_eval_gpu_s;
      valid = std::isfinite(mcc) && mcc > 0.0 && !forced_invalid;
      if (merged && valid && cand_err != MVBA_OK) throw StatusErr{cand_err, device_error_text(cand_err)};
      if (merged && !valid) {  // the speculative candidate moved the parameters
        // prep() starts a new evaluation generation: the candidate's error
        // word (stamped with the old one) is stale from here on
        set_params_from(S_->x);
        prep();
      }
    }
    sum->linear_solver_time_s += now_s() - ts - m_eval_gpu_s;
    sum->eval_time_s += m_eval_gpu_s;
    static const bool trace = std::getenv("MVBA_SOLVER_TRACE") && std::getenv("MVBA_SOLVER_TRACE")[0] == '1';
    if (trace)
      std::fprintf(stderr,
                   "mvba trace: it %d cg status %d iters %d | model change %.6e (|Jd|^2 %.6e, gp'dp %.6e, "
                   "gc'dc %.6e) | gmax %.3e radius %.3e\n",
                   iteration, cgr.status, cgr.iters, mcc, last_mc_[0], last_mc_[1], last_mc_[2], gmax, radius);
    if (!valid) {
      // HandleInvalidStep
      if (++invalid >= o_.max_num_consecutive_invalid_steps) {
        std::snprintf(buf, sizeof(buf),
                      "Number of consecutive invalid steps more than Solver::Options::max_num_consecutive_invalid_steps: %d",
                      o_.max_num_consecutive_invalid_steps);
        finish(MVBA_FAILURE, buf);
        break;
      }
      radius /= decrease;
      decrease *= 2.0;
      successful = false;
      sum->num_unsuccessful_steps++;
      row(x_cost, 0.0, 0.0, 0.0, cgr.iters, now_s() - it0);
      continue;
    }
    invalid = 0;
    bool relinearized = false;
    const double te = now_s();
    if (bounded_) {
      // g'delta: model change = -(g'delta + |J delta|^2/2) has g'delta in it; recompute directly
      const double gtd = dot_global(S_->G, S_->delta);
      armijo(x_cost, gtd, &relinearized);
    }
    // ComputeCandidatePointAndEvaluateCost (merged: already read with the step)
    double cand = m_cand;
    if (!merged) {
      HCHK(mvba_launch_plus(nc, S_->x, S_->delta, S_->lo, S_->hi, S_->xn, s_));
      set_params_from(S_->xn);
      cand = cost();
    }
    if (!std::isfinite(cand)) cand = std::numeric_limits<double>::max();
    sum->eval_time_s += now_s() - te;
    const double step_norm = merged ? std::sqrt(m_step2) : std::sqrt(step_norm2());
    auto restore_x = [&]() {
      set_params_from(S_->x);
      prep();
    };
    if (step_norm <= o_.parameter_tolerance * (x_norm + o_.parameter_tolerance)) {
      std::snprintf(buf, sizeof(buf), "Parameter tolerance reached. Relative step_norm: %e <= %e.",
                    step_norm / (x_norm + o_.parameter_tolerance), o_.parameter_tolerance);
      finish(MVBA_CONVERGENCE, buf);
      restore_x();
      break;
    }
    const double change = x_cost - cand;
    if (trace)
      std::fprintf(stderr, "mvba trace:   step %.6e (x %.6e) cost %.17g -> %.17g change %.6e ratio %.6e\n",
                   step_norm, x_norm, x_cost, cand, change, change / mcc);
    if (std::fabs(change) <= o_.function_tolerance * x_cost) {
      std::snprintf(buf, sizeof(buf), "Function tolerance reached. |cost_change|/cost: %e <= %e",
                    std::fabs(change) / x_cost, o_.function_tolerance);
      finish(MVBA_CONVERGENCE, buf);
      restore_x();
      break;
    }
    const double ratio = change / mcc;
    if (ratio > o_.min_relative_decrease) {
      // HandleSuccessfulStep: x = candidate, re-linearize there (cost() ran the
      // prep kernel at the candidate: its records are current)
      std::swap(S_->x, S_->xn);
      if (merged) {
        // |x|, the linearization at x (records current: cost() ran K0 there) and
        // the projected-gradient max norm, read back together
        tl = now_s();
        norm2_enqueue(S_->x, 5, 6);
        linearize_enqueue(true, 1);
        grad_max_enqueue(0);
        const double* hs = fetch_checked(7);
        x_norm = std::sqrt(hs[5] + hs[6]);
        x_cost = hs[1];
        gmax = hs[0];
        sum->linearize_time_s += now_s() - tl;
      } else {
        x_norm = std::sqrt(norm2_compact(S_->x));
        tl = now_s();
        x_cost = linearize(true);
        sum->linearize_time_s += now_s() - tl;
        gmax = grad_max_norm();
      }
      radius = std::min(o_.max_trust_region_radius,
                        radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * ratio - 1.0, 3)));
      decrease = 2.0;
      successful = true;
      sum->num_successful_steps++;
      row(x_cost, change, step_norm, ratio, cgr.iters, now_s() - it0);
    } else {
      // HandleUnsuccessfulStep
      radius /= decrease;
      decrease *= 2.0;
      successful = false;
      sum->num_unsuccessful_steps++;
      restore_x();
      if (relinearized) linearize();
      row(cand, change, step_norm, ratio, cgr.iters, now_s() - it0);
    }
  }
  HCHK(hipStreamSynchronize(s_));
  sum->num_iterations = iteration;
  sum->cg_graph_launches = graph_launches_;
  sum->final_cost = x_cost;
  sum->total_time_s = now_s() - t0;
  if (cg_timing() && tm_.solves)
    std::fprintf(stderr,
                 "mvba cg timing: %d solves, %d CG iterations (%d enqueued, %d batches) | us per solve: prologue "
                 "(damping, prec, rhs, cg start) %.1f, back-substitution %.1f | us per enqueued iteration: "
                 "enqueue %.1f, wait %.1f | loop us per CG iteration %.1f | graph launches %d\n",
                 tm_.solves, tm_.iters, tm_.enqueued, tm_.batches, 1e6 * tm_.rhs / tm_.solves, 1e6 * tm_.backsub / tm_.solves,
                 1e6 * tm_.enqueue / std::max(tm_.enqueued, 1), 1e6 * tm_.wait / std::max(tm_.enqueued, 1),
                 1e6 * (tm_.enqueue + tm_.wait) / std::max(tm_.iters, 1), graph_launches_);
}

}  // namespace

extern "C" {

void mvba_solver_default_options(mvba_solver_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->max_num_iterations = 50;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->min_relative_decrease = 1e-3;
  o->eta = 1e-1;
  o->min_linear_solver_iterations = 0;
  o->max_linear_solver_iterations = 500;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->use_loss = 0;
  o->robust_threshold = 0.0;
}

// One non-blocking stream per device for solves called on the null stream,
// created on first use and kept for the process's lifetime (handles come and go
// per pass in the CLI; a stream per handle would be created and destroyed with
// each). The sanitizer build's failure with per-handle streams
// (profiles/r05/r05h/san_cli_g0_r05h.log:124-153): at exit, libamdhip64's own
// static destructors (__cxa_finalize) free HSA runtime objects; ASan's
// quarantine, taking that free, recycles older quarantined chunks, and among
// them were device allocations made through ASan's device allocator and
// released earlier by hipStreamDestroy (a stream's queue memory). ASan had by
// then marked the device runtime unloaded, so DeviceAllocator::Deallocate
// failed its CHECK. No object of ours frees anything after the runtime
// unloads; what matters is that no destroyed stream's device memory sits in
// the quarantine when HIP tears down, which one stream per process ensures.
hipStream_t solver_stream(int device) {
  static std::mutex m;
  static std::vector<hipStream_t> streams;
  std::lock_guard<std::mutex> lk(m);
  if ((int)streams.size() <= device) streams.resize((size_t)device + 1, nullptr);
  if (!streams[(size_t)device] &&
      hipStreamCreateWithFlags(&streams[(size_t)device], hipStreamNonBlocking) != hipSuccess) {
    streams[(size_t)device] = nullptr;
    throw HipErr{hipErrorOutOfMemory, "hipStreamCreateWithFlags"};
  }
  return streams[(size_t)device];
}

mvba_status mvba_solve(mvba_handle* h, const mvba_solver_options* o, mvba_solver_summary* summary,
                       void* stream) {
  if (!h || !o || !summary) return MVBA_E_INVALID;
  std::memset(summary, 0, sizeof(*summary));
  if (!h->lin_ok) return h->fail(MVBA_E_INVALID, h->lin_err);
  if (!h->params_set) return h->fail(MVBA_E_INVALID, "parameters were not set (mvba_set_params)");
  if (o->use_loss && !(o->robust_threshold > 0.0)) return h->fail(MVBA_E_INVALID, "The robust threshold must be positive.");
  if (o->max_num_iterations < 0 || o->max_linear_solver_iterations < 1 || !(o->initial_trust_region_radius > 0.0))
    return h->fail(MVBA_E_INVALID, "invalid solver options");
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  // the library's own stream (a null-stream caller): a failed solve drains it
  // before returning, so no kernel queued before the failure still writes the
  // parameters or solver buffers behind the caller's next null-stream call
  // (a non-blocking stream does not order against the null stream)
  hipStream_t lib_stream = nullptr;
  auto drain = [&]() {
    if (lib_stream) (void)hipStreamSynchronize(lib_stream);
    (void)hipGetLastError();
  };
  try {
    if (!h->solver) h->solver = alloc_state(h);
    // A caller on the null stream gets the handle's own stream: the CG loop's
    // graphs cannot be captured on the null stream. The solve is host-
    // synchronous anyway (it ends with a stream sync); it starts after all
    // earlier device work, so it sees the caller's null-stream writes.
    // (single-rank and RCCL-sharded solves: shards of one process on the
    // local communicator keep the caller's stream, where a device-wide sync
    // could wait on a peer shard's pending exchange)
    hipStream_t st = (hipStream_t)stream;
    static const bool own = !(std::getenv("MVBA_OWN_STREAM") && std::getenv("MVBA_OWN_STREAM")[0] == '0');
    // (an RCCL-sharded solve too: one process per device, so the device-wide
    // sync waits only for this rank's work, and its CG runs can be captured
    // with the exchange inside; r06a: on the null stream every sharded CG
    // kernel was launched eagerly)
    const bool rccl = o->allreduce == &mvba_comm_allreduce &&
                      mvba_comm_capturable((const mvba_comm*)o->allreduce_user);
    if (!st && (!o->allreduce || rccl) && own) {
      HCHK(hipDeviceSynchronize());
      st = solver_stream(h->device);
      lib_stream = st;
    }
    Solver sv(h, *o, st);
    // K2 writes the CG passes' per-slot records for the duration of the solve
    struct ObsxScope {
      mvba_handle* h;
      ~ObsxScope() { h->lin_obsx = nullptr; }
    } scope{h};
    h->lin_obsx = sv.obsx_records();
    sv.run(summary);
  } catch (const HipErr& e) {
    drain();
    std::snprintf(summary->message, sizeof(summary->message), "HIP error");
    summary->termination_type = MVBA_FAILURE;
    return h->hip_fail(e.e, e.where);
  } catch (const StatusErr& e) {
    drain();
    summary->termination_type = MVBA_FAILURE;
    std::snprintf(summary->message, sizeof(summary->message), "%s", e.msg.c_str());
    return h->fail(e.st, e.msg);
  } catch (const std::bad_alloc&) {
    drain();
    return h->fail(MVBA_E_INVALID, "host allocation failed");
  }
  return MVBA_OK;
}

mvba_status mvba_get_params(mvba_handle* h, double* packed) {
  if (!h || !packed) return MVBA_E_INVALID;
  if (hipSetDevice(h->device) != hipSuccess) return h->fail(MVBA_E_HIP, "hipSetDevice failed");
  hipError_t e = hipMemcpy(packed, h->d_params, (size_t)h->nparams * sizeof(double), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return h->hip_fail(e, "mvba_get_params");
  return MVBA_OK;
}

}  // extern "C"
