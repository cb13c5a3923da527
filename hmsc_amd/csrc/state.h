// Device-resident state of one Hmsc chain (or one species shard of a chain).
//
// HBM layout (all fp64 column-major like R unless noted):
//   Z        ny x ns_loc          latent responses (the only large mutable array)
//   Ycode    ny x ns_loc  int8    0 / 1 / -1(NA)           (probit cells)
//   Yval     ny x ns_loc          YScaled (only if non-probit species exist)
//   X        ny x nc              XScaled
//   BL       K x ns_loc           [Beta; Lambda_1; ...; Lambda_nr]   (K = nc + sum nf_r)
//   Psi      NF x ns_loc          [Psi_1; ...; Psi_nr]               (NF = sum nf_r)
//   Delta    NF                   [Delta_1; ...]
//   Eta_r    np_r x nf_r          per level, column-major
// Live K/NF change only through updateNf (transient), which repacks on the host;
// buffers are allocated at nfMax so no reallocation ever happens.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <memory>
#include <vector>

#include "../../include/hmsc_amd.h"
#include "rng.h"

namespace hmsc {

struct Level {
  int np = 0, nf = 0, nfmax = 0, nfmin = 0;
  // factors this level's buffers hold: min(nfMax, K cap - nc) -- Eta storage, record slots;
  // and the factors its spatial workspace is laid out for now (grown with nf, spatial.hip)
  int nfcap = 0, nf_alloc = 0;
  double nu = 3, a1 = 50, b1 = 1, a2 = 50, b2 = 1;
  double* Eta = nullptr;        // np x nfmax storage, live np x nf (ld = np)
  int* Pi = nullptr;            // ny, 0-based unit of each row
  int* unit_ptr = nullptr;      // np+1 CSR over rows of each unit
  int* unit_rows = nullptr;     // ny
  int* Alpha = nullptr;         // nfmax (host mirror in State::h_alpha)
  int uniform_n = 0;            // common row count of every unit (0 if they differ)
  // spatial "Full" level (spatial.hip): alphapw grid of R/computeDataParameters.R:53-81
  bool spatial = false;
  int nalpha = 0;
  double* alphapw = nullptr;    // nalpha x 2
  double* iWg = nullptr;        // np x np x nalpha
  double* RiWg = nullptr;       // np x np x nalpha (upper triangular; lower for NNGP / GPP)
  int riw_lower = 0;            // RiWg lower: NNGP's Vecchia factor, GPP's / the device-built Full grid's chol(W)^-1
  double* detWg = nullptr;      // nalpha
  double* AlphaD = nullptr;     // nfmax: 1-based grid index of each factor (recorded)
  double* spWork = nullptr;     // dense (np nf)^2 Eta system + Alpha likelihoods
  // 'GPP' level in R's low-rank form (spatial.hip, R/computeDataParameters.R:138-194)
  bool gpp = false;
  int nK = 0;
  double* idDg = nullptr;       // np x nalpha
  double* idDW12g = nullptr;    // np x nK x nalpha
  double* Fg = nullptr;         // nK x nK x nalpha
  double* iFg = nullptr;        // nK x nK x nalpha
  // 'NNGP' level in the sparse Vecchia form (spatial.hip, R/computeDataParameters.R:82-136):
  // RiW_g = D_g^-1/2 (I - A_g), A_g[i, nb(i, k)] over the nnK nearest earlier units
  bool nngp = false;
  int nnK = 0;                  // neighbours per unit (rL$nNeighbours)
  int* nnIdx = nullptr;         // nnK x np: earlier neighbours of unit i (ascending), -1 padded
  double* nnA = nullptr;        // nalpha x nnK x np: Vecchia coefficients A_g[i, nb(i, k)]
  double* nnD = nullptr;        // nalpha x np: conditional variances D_g[i]
  int* nnPerm = nullptr;        // np: unit at each position of the factorization order (RCM)
  int* nnPos = nullptr;         // np: position of each unit
  int* nnChPtr = nullptr;       // np + 1: CSR of the rows whose support {i} + nb(i) holds the unit
  int* nnCh = nullptr;          // entries i (nnK + 1) + slot, slot 0 = the unit itself (B = 1), ascending i
  int nnBwUnits = 0;            // bandwidth of the precision in units (RCM order)
  int nnAssembledN = 0;         // size of the last assembled system (its band layout zeroed for it)
  // covariate-dependent level (hmsc_model etaShare / xScale): the level whose units and Eta
  // this one shares (eta_owner < this index: Eta aliases the owner's buffer), the covariate
  // column scaling its XEta columns (np, unit order), and -- on the owner -- the levels of
  // its group (xgroup consecutive levels from it)
  int eta_owner = -1;
  double* xs = nullptr;
  int xgroup = 1;
  bool eta_alias() const { return eta_owner >= 0; }
};

struct State {
  // dims
  int ny = 0, ns = 0, nc = 0, nt = 0, nr = 0;
  int sp0 = 0, nsl = 0;          // species shard [sp0, sp0+nsl)
  int rank = 0, nranks = 1;
  int device = 0;
  uint32_t mask = HMSC_UP_ALL;
  Key key{0, 0};
  int noise_mode = 0;
  bool has_na = false;           // any NA in the local Y
  bool any_normal = false;       // any family==1 species (local)
  bool any_var = false;          // any species with estimated variance (distr[,2]==1)
  bool any_poisson = false;
  bool any_xs = false;           // a covariate-dependent level (Level::xs): general updateEta path
  bool all_probit = true;
  bool isigma_fixed_one = true;  // all probit and iSigma never set from outside: iSigma == 1
  int K = 0, NF = 0, Kmax = 0, NFmax = 0;
  double f0 = 0;
  Level lev[HMSC_MAX_LEVELS];

  hipStream_t stream = nullptr, copy_stream = nullptr;
  // side stream: updateGammaV, Gamma2's iV-only algebra and updateLambdaPriors of sweep t
  // only feed sweep t+1, so they overlap updateEta / updateZ of sweep t
  hipStream_t side = nullptr, side2 = nullptr;  // side: GammaV + Gamma2 prep; side2: LambdaPriors
  // a captured recorded sweep asks updateZ's slab-sum launch to carry the record pack (part 1)
  bool pack_req = false, pack_done = false;
  hipEvent_t ev_bl = nullptr, ev_side = nullptr, ev_side2 = nullptr;
  int side_pending = 0;          // bit 0: side has unjoined work (ev_side), bit 1: side2 (ev_side2)
  // co-launched sweep (see launch_side_fused): only the GammaV algebra stays on `side`; its
  // Philox sweep counter is snapshotted into d_iter_side by the launch that forks it, so the
  // main stream may advance d_iter for the next sweep while it runs
  bool side_fused = false;
  bool crw_fresh = false;   // the last Gamma2 + BetaLambda launch formed the fused Eta constants
  bool tail_defer = false;  // ... with its reductions left to the Eta launch (EF_DEFER)
  // ... and its BetaLambda tail also formed GammaV's and LambdaPriors' species partials (gvt),
  // which the side chain reads instead of post_bl_kernel's
  bool tail_gv = false;
  // HMSC_SIDE_PARTIALS=1 (read at create): the species partials always from post_bl_kernel on
  // the side stream, forked on the device at the tails flag -- the fused launch ends ~5 us
  // sooner, but the side work beside Eta and z costs them about as much (same 1000-step rate)
  // and a replay's first sweeps wait longer for it (20-step line ~2 % lower)
  bool side_partials = false;
  // kernel record copies (HMSC_KERNEL_COPY, kernels.hip rec_copy_kernel): graph replays' packs
  // raise pack_flags and a copy kernel per sample moves it to the host ring
  bool kcopy = false;
  int kcopy_max = 8;               // ... for the recorded graphs of at most this many sweeps
  bool cap_kcopy = false;          // the capture in progress packs with flags
  uint64_t* pack_flags = nullptr;  // [3 parts][ring_slots]
  int* pack_ticket = nullptr;      // [3 parts, copy kernel]
  uint32_t run_nonce = 0;          // desc[4]: flags of an earlier run never match
  double* host_rec_dev = nullptr;  // the pinned host ring's device address
  int cap_pack_mask = 0;           // pack parts captured since the last reset (capture_sweeps)
  bool long_tail = false;   // HMSC_LONG_TAIL=1: a recorded run's last replay not split into single sweeps
  // HMSC_FIRST_REPLAY=k: a run's first replay at most k sweeps (0, the default: no limit).  It
  // takes the side-node dispatch delay of a big first replay away (device span of a 20-sweep
  // run -25 us), but the 16-sample copy of the following replay then trails the run (its
  // 20-step line 5,260 -> 5,110 sweeps/s same box)
  int first_replay = 0;
  // graph sweeps after the first of a capture (cap_sweep > 0): the side work is not forked
  // from the main stream nor joined into it by graph edges (each a ~5-6 us cross-queue gap on
  // the critical path) but synchronised by device flags: its first launch waits for the fused
  // launch's tails (gbl_sync[2]), and the next fused launch waits for its side_sync flags
  int cap_sweep = -1;
  bool edge_free = true;    // (HMSC_SIDE_EDGES=1: graph edges everywhere)
  // edge_free for the capture in progress / the graphs held: only while this chain is the one
  // live chain on its device in the process.  Device-side joins need the main and side streams
  // on separate hardware queues; the streams of several chains (nParallel > 1 on one GPU) can
  // share the few queues and wait on each other in a cycle, so their graphs keep
  // graph edges, and graphs captured edge-free are rebuilt once a second chain appears.
  bool edge_free_now = false, graph_edge_free = false;
  bool counted_live = false;  // counted in capi.cpp's live chains of its device
  int g2bl_last_tail = -1, g2bl_last_nb = 0;  // the last fused Gamma2 + BetaLambda launch's layout (debug_get "g2bl")
  bool side_gated = false;  // the last slab launch waited for the side chain's flags (SideGate)
  bool side_tail = false;   // the last side chain raises side_sync (the next fused launch may join it on the device)
  // the capture in progress forked the side stream at the graph's root, so its first sweep's
  // side work waits for the tails flag on the device too (no edge from the fused launch)
  bool side_root = false;
  bool psi_side = true;     // the last sweep's psi draws ran on the side stream (post_bl_kernel), not in the tail
  int* side_sync = nullptr;      // [GammaV, delta chain per level ..., Gamma2 prep, (slot SIDE_ARB_SLOT) the
                                 // sharded Eta solve's all-reduce-B flag]: epoch of the sweep
  bool shard_dev = false;        // this sharded sweep joins and forks its side chain on the device (sweep_sharded)
  bool g2s_slab_req = false;     // sweep_sharded: updateZ's slab launch may form all-reduce A's sums ...
  bool g2s_slab = false;         // ... and did (shard_g2_stats then only all-reduces)
  double* gvt = nullptr;         // the BetaLambda tail's GammaV / psi partial tiles
  int gvt_ld = 0;
  double* Gamma_side = nullptr;  // GammaV's Gamma, for the side stream's record pack
  uint32_t* d_iter_side = nullptr;
  double* gv_part = nullptr;     // GammaV species partials (not shared with Gamma2's ABpart)

  // model (device)
  double *X = nullptr, *Tr = nullptr, *Yval = nullptr, *Yraw = nullptr;
  int8_t* Ycode = nullptr;
  uint64_t* Ybits = nullptr;     // ceil(nsl / 32) x ny: the same codes + 1, 2 bits per species (z kernel)
  double* logtab = nullptr;      // z_log_table: the z kernel's table log (ZLOG_N x ZLOG_W)
  int* fam = nullptr;            // ns_loc family code
  int* varest = nullptr;         // ns_loc distr[,2]
  double *V0 = nullptr, *iUGamma = nullptr, *mGamma = nullptr, *UGammaL = nullptr, *UGamma = nullptr;
  double* geWork = nullptr;      // updateGammaEta workspace (gamma_eta.hip), only if that updater is on
  size_t geWork_doubles = 0;     // its size (grown with the levels' nf)
  double *aSigma = nullptr, *bSigma = nullptr;
  double *XX = nullptr, *TT = nullptr, *V0g = nullptr, *V0gXXV0g = nullptr, *iV0 = nullptr;
  double* V0inv = nullptr;       // V0^-1 (initial riwish draw)
  double* iUmG = nullptr;        // iUGamma %*% mGamma
  double* V0gXX = nullptr;       // Gamma2 prior covariance times X'X
  double* g2prep = nullptr;      // Gamma2 iV-only matrices [A1|B1|TR|LS]
  double* scratch2 = nullptr;    // side-stream scratch
  bool g2prep_valid = false;
  int* na_cols = nullptr;        // local species with any NA
  int* na_index = nullptr;       // nsl: row of species j in Gna, or -1
  int n_na_cols = 0;
  int* na_rows = nullptr;        // rows with any NA in the whole Y (every rank of a sharded chain: the same rows)
  int8_t* row_na = nullptr;      // ny: 1 if the row has an NA
  int* row_slot = nullptr;       // ny: index into na_rows, or -1
  int n_na_rows = 0;
  int* dev_flags = nullptr;      // device error flags (Cholesky failures)
  int* gbl_sync = nullptr;       // gamma2_bl_kernel's in-launch handshake [ticket, Gamma epoch, tails epoch, error]
  std::vector<int> h_na_cols;

  // chain state (device)
  double *Z = nullptr, *BL = nullptr, *Psi = nullptr, *Delta = nullptr;
  double *Gamma = nullptr, *iV = nullptr, *iSigma = nullptr;
  double* rho = nullptr;          // updateRho grid index, 1-based (R's rho), as a double

  // phylogeny (hM$C != NULL, phylo.hip): spectral form of computeDataParameters' Qg grid
  bool phylo = false;
  int nrho = 0;
  int phNmax = 0;                // K * ns the dense BetaLambda workspace holds
  double* phU = nullptr;         // ns x ns eigenvectors of C
  double* phWinv = nullptr;      // nrho x ns  1 / q_g,i
  double* phRbase = nullptr;     // nrho  log(rhopw[,2]) - nc/2 logdet Q_g
  double* phTt = nullptr;        // ns x nt  U^T Tr
  double* phBt = nullptr;        // nc x ns  Beta U
  double* phEt = nullptr;        // nc x ns  Beta U - Gamma Tt^T
  double* phTTw = nullptr;       // nt x nt  Tr^T iQ Tr
  double* phWork = nullptr;      // dense BetaLambda / Rho workspace

  // per-sweep workspaces
  double* XEta = nullptr;        // ny x Kmax    [X, Eta_1[Pi_1], ...] materialised per Eta update
  bool xeta_valid = false;
  // G's Eta rows from the fused Eta pass' tile partials not reduced yet: the next updateZ
  // launch reduces them on extra workgroups (z_kernel.h), any other reader of G first calls
  // flush_g (kernels.hip)
  bool g_pending = false;
  int g_ntile = 0, g_nf = 0;
  double* XZ = nullptr;          // K x ns_loc   XEta^T (Yx o Z)
  double* G = nullptr;           // Kmax x Kmax  XEta^T XEta
  double* ZTr = nullptr;         // ny x nt      Z Tr (local species)
  double* XZ_part = nullptr;     // nchunk x K x ns_loc
  // the next sweep's BetaLambda noise and psi gamma variates, drawn ahead by the Eta launch
  // (kernels.hip bl_predraw_body): [species][64] (lane k < K: xi; 32 + f: psi's gamma), and
  // the (sweep, K) they were drawn for
  double* bl_pre = nullptr;
  int* bl_pre_tag = nullptr;
  double* G_part = nullptr;      // nchunk x Kmax^2
  double* ZTr_part = nullptr;    // ntile_j x ny x nt
  double* Gna = nullptr;         // n_na_cols x Kmax^2 masked grams
  double* ZL = nullptr;          // ny x NFP   Z * (Lambda diag(iSigma))^T, all levels
  double* ZL_part = nullptr;     // zl_split x ny x NFP
  double* CR = nullptr;          // Kmax x NFmax  BL diag(iSigma) Lambda_all^T
  double* CR_part = nullptr;     // species-block partials of CR
  double* LS = nullptr;          // NFmax x ns_loc  Lambda_all diag(iSigma) (fused Eta kernel)
  double* crw_part = nullptr;    // the fused Eta constants' partial tiles (kernels.hip crw_body / crw_tail)
  int* crw_ticket = nullptr;     // [crw_kernel, crw_tail's groups, crw_tail's per-group tickets, crw_flag]
  int* crw_flag = nullptr;
  // XZ left as updateZ's chunk partials (their count; 0: s.XZ holds it): the fused Gamma2 +
  // BetaLambda launch sums its columns where it reads them, everything else calls flush_xz
  int xz_parts = 0;       // epoch of the sweep whose CR / W a deferred tail published (EF_DEFER)
  double* etaW = nullptr;        // 16 x 16  L^-1 of Q = I + Lambda diag(iSigma) Lambda^T (fused Eta kernel)
  double* Msmall = nullptr;      // per-level masked row grams (NA rows)
  double* scratch = nullptr;     // single-workgroup updaters
  double* psi_rs = nullptr;      // psi-lambda^2 row-sum partials
  double* ABpart = nullptr;      // GammaV species-partials
  double* dbg_prec = nullptr;    // optional debug: per-species precisions
  bool zt_valid = false;         // XZ/G/ZTr computed for the current Z and Eta
  int nchunk = 0, ntile_j = 0, zl_split = 0, NFP = 0;
  size_t scratch_doubles = 0;
  size_t scratch2_doubles = 0;  // Gamma2's prep working set, then its final stage's arrays past 64 KB

  // recording ring
  double* ring = nullptr;
  int ring_slots = 0;
  size_t slot_doubles = 0;
  double* host_rec = nullptr;    // pinned host ring (ring_slots slots)
  uint64_t* copied_host = nullptr;  // fine-grained pinned counter: samples whose D2H copy landed
  uint64_t* copied_dev = nullptr;   // its device address
  std::shared_ptr<struct UnpackPool> unpack_pool;
  int* trsv_sync = nullptr;  // the dense handshake block (DENSE_SYNC_INTS ints, zeroed): sync-free solves, fused panel

  // per-sweep hipGraph (single rank, no updateNf): captured once, replayed every sweep; the
  // kernels read the Philox sweep counter from d_iter, which the graph's first node advances
  uint32_t* d_iter = nullptr;          // the Philox sweep counter captured kernels read (a slot of d_iters)
  uint32_t* d_iters = nullptr;         // one counter per captured sweep; a replay's last kernel advances them
  bool capturing = false;
  bool use_graph = true;
  bool graph_dirty = true;
  int graph_K = -1, graph_NF = -1;
  // gx[rec][k]: 2^k consecutive sweeps (rec: each followed by the record pack), k = 0 ..
  // log2(graph_sweeps); a run of n sweeps replays its binary decomposition, largest first
  static constexpr int GRAPH_LEVELS = 7;  // up to 64 sweeps per replay
  hipGraphExec_t gx[2][GRAPH_LEVELS] = {};
  int gx_pack_mask[2][GRAPH_LEVELS] = {};  // kcopy: the pack parts every recorded sweep of the graph raises (-1: mixed)
  // The first sweep of a replay's side work (side chain [+ record pack part 2]) runs outside
  // the graph: a graph launch submits its side-stream nodes only after all its main-stream
  // nodes (~16 us of host time per sweep), so that sweep's side chain started late and the
  // next sweep's fused launch waited for it.  capture_sweeps keeps it as a closure per graph
  // (ext_side, launched on the side stream ahead of the graph by replay_sweeps) instead.
  std::function<void()> ext_pending;                // built while capturing sweep 0
  std::function<void()> ext_side[2][GRAPH_LEVELS];  // per graph in gx
  uint32_t* d_ext_iter = nullptr;                   // the external side work's sweep counter
  hipEvent_t ev_ext = nullptr;                      // after it: the record copy waits on it
  hipEvent_t ev_ext_go = nullptr;                   // the replay's start, which it waits behind
  bool ext_launched = false;
  bool single_stream = false;          // HMSC_SINGLE_STREAM: no side-stream overlap (diagnostic)
  int graph_sweeps = 4;                 // sweeps per replay, a power of two (HMSC_GRAPH_SWEEPS)
  uint32_t dev_iter_next = 0;           // the sweep the device's d_iters slots already hold (valid_iters)
  bool valid_iters = false;
  int32_t* d_rec_desc = nullptr;        // {iter0, transient, thin, samples} of the current run
  hipEvent_t ev_graph = nullptr;        // after a recording replay: the copy stream waits on it
  int eager_streak = 0;          // eager steady sweeps since the graph was invalidated

  // live launch timing of the timed kernels (common.h kt_record): per-sweep-slot first
  // start / last finish wall-clock ticks, KT_N blocks of 2 * KT_SLOTS
  unsigned long long* d_kt = nullptr;
  bool kt_on = false;

  // live kernel timing (HIP events on this chain's stream), id -> launches
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_ev[10];

  // RCCL (species-sharded chain), or a host transport (hmsc_create_sharded_host)
  void* comm = nullptr;
  double* allreduce_buf = nullptr;
  hmsc_allreduce_fn host_allreduce = nullptr;
  void* host_allreduce_ctx = nullptr;
  std::vector<double> host_ar_buf;

  // ---- species-sharded chain (kernels.hip "species-sharded sweep", capi.cpp sweep_sharded).
  // A sharded chain (nranks > 1, or a 1-rank chain created with a communicator or a host
  // transport) reduces its cross-species sums in exactly two all-reduces per sweep:
  //   A (after updateZ, for the next sweep's updateGamma2): ar_a = [X^T Z Tr (nc nt) |
  //     Lambda_all Tr (NF nt) | #(iSigma != 1)]   (R/updateGamma2.R:36,46)
  //   B (after updateBetaLambda): ar_b = [ZL = Z (Lambda diag(iSigma))^T (ny NF, site-major) |
  //     CR = BL diag(iSigma) Lambda^T (K x NF, ld K) | GammaV's E E^T, B Tr (nc^2 + nc nt) |
  //     sum_j psi lambda^2 (NF) | NA rows: CR masked to the row's observed species
  //     (n_na_rows x K x NF)]   (R/updateEta.R:45-55,59-70, R/updateGammaV.R:16-18,
  //     R/updateLambdaPriors.R:22-32)
  // Everything downstream of a sum (Gamma, iV, Delta, Eta) is drawn redundantly on every
  // rank from the same Philox counters, so the ranks' copies stay bit-identical.
  bool sharded = false;
  bool any_na_global = false;    // any NA in the whole Y (the fusion decisions of every rank agree)
  double* ar_a = nullptr;
  double* ar_b = nullptr;
  double* ar_host = nullptr;     // pinned host staging of the host transport (max of A, B)
  size_t ar_host_doubles = 0;
  int* shard_ticket = nullptr;   // [g2 stats ticket, spare]: zero between launches
  bool g2s_valid = false;        // ar_a holds the reduced Gamma2 sums of the current Z, BL, iSigma
  // debug counters (hmsc_debug_get "ar_calls"): collectives issued / executed and their doubles;
  // the all-reduces a captured sweep contains (graph replays add ar_per_graph_sweep per sweep)
  uint64_t ar_calls = 0, ar_doubles = 0;
  int ar_in_capture = 0, ar_per_graph_sweep = -1;
  // host transport inside graph capture: a sweep is captured as segments split at its
  // all-reduces (the host sums between them); cap_segs collects them during the capture
  struct Seg {
    hipGraphExec_t g = nullptr;
    size_t ar_n = 0;             // doubles of ar_host to all-reduce after this segment (0: none)
    double* ar_dev = nullptr;    // (the device buffer the next segment copies the sum back into)
  };
  std::vector<std::pair<hipGraph_t, size_t>>* cap_segs = nullptr;
  std::vector<Seg> gseg[2];      // [with record]: one sweep of a host-transport sharded chain

  std::vector<int> h_nf() const {
    std::vector<int> v(nr);
    for (int r = 0; r < nr; ++r) v[r] = lev[r].nf;
    return v;
  }
  int loff(int r) const {  // row offset of level r inside BL
    int o = nc;
    for (int q = 0; q < r; ++q) o += lev[q].nf;
    return o;
  }
  int foff(int r) const {  // row offset of level r inside Psi / Delta
    int o = 0;
    for (int q = 0; q < r; ++q) o += lev[q].nf;
    return o;
  }
  void refresh_dims() {
    NF = 0;
    for (int r = 0; r < nr; ++r) NF += lev[r].nf;
    K = nc + NF;
  }
};

enum ProfId {
  PROF_Z = 0, PROF_ZL = 1, PROF_BL = 2, PROF_ETA_UNIT = 3, PROF_SWEEP = 4,
  PROF_ETA_SP = 5,  // spatial updateEta (assembly + blocked Cholesky + solves)
  PROF_CHOL = 6,    // the blocked Cholesky inside it
  PROF_ALPHA = 7,   // updateAlpha (grid quadratic forms + draw)
  PROF_GE = 8,      // updateGammaEta (all levels)
  PROF_RHO = 9,     // updateRho
  PROF_N = 10
};
static_assert(PROF_N <= 10, "State::prof_ev holds 10 profile ids");

struct ProfScope {  // records a start/stop event pair around one launch when profiling is on
  State& s;
  int id;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(State& st, int i) : s(st), id(i) {
    if (s.prof) {
      (void)hipEventCreate(&a);
      (void)hipEventCreate(&b);
      (void)hipEventRecord(a, s.stream);
    }
  }
  ~ProfScope() {
    if (s.prof) {
      (void)hipEventRecord(b, s.stream);
      s.prof_ev[id].emplace_back(a, b);
    }
  }
};

// launchers implemented in kernels.hip
void launch_init(State& s);
void launch_update_z(State& s, uint32_t iter, bool use_raw_y);
void launch_zt_refresh(State& s);
int z_resident_slots(const State& s);
int z_xeta_cols_for(int Kmax);  // XEta columns the z kernel reads (zdraw.hip)
void flush_xz(State& s);        // reduce XZ from its chunk partials if they are pending (kernels.hip)
void ext_add_record(State& s);  // add record pack part 2 to the external first-sweep side work (kernels.hip)
void launch_xeta(State& s);
void flush_g(State& s);
// SideGate: the slab launch after updateZ waits (one extra workgroup) for the flags of this
// sweep's side chain that the next sweep's fused Gamma2 + BetaLambda launch would otherwise
// poll at its start (kernels.hip side_gate_next); n = 0: no gate
struct SideGate {
  const int* flags = nullptr;
  int n = 0;
  uint32_t iter = 0;
  const uint32_t* iter_dev = nullptr;
  int* err = nullptr;
};
SideGate side_gate_next(State& s, uint32_t iter);
// g2s (a sharded chain's sweep, p0 = updateZ's XZ chunk partials): all-reduce A's species sums
// formed in the same launch (g2_stats_body)
void launch_slab_sum2(const double* p0, double* o0, int64_t n0, int np0, const double* p1, double* o1, int64_t n1,
                      int np1, hipStream_t st, SideGate gate = SideGate{}, State* g2s = nullptr);
// the same with the main-stream record pack (part 1) of a captured recorded sweep appended
void launch_slab_sum2_pack(State& s, const double* p0, double* o0, int64_t n0, int np0, const double* p1, double* o1,
                           int64_t n1, int np1, SideGate gate = SideGate{}, State* g2s = nullptr);
void launch_beta_lambda(State& s, uint32_t iter);
void launch_gamma_v(State& s, uint32_t iter, hipStream_t st);
void launch_gamma2(State& s, uint32_t iter);
bool gamma2_bl_fusion_ok(const State& s);
void launch_gamma2_bl(State& s, uint32_t iter);  // updateGamma2 + updateBetaLambda in one launch
int live_chains_on(int device);                  // chains created and not destroyed on a device (capi.cpp)
// a species-sharded chain on RCCL: a recorded graph sweep packs its main-stream quantities in
// updateZ's slab launch and the side chain's (Gamma, iV, Delta) on the side stream after it,
// so no pack launch waits behind all-reduce A on the main stream (capi.cpp record_after_sweep)
inline bool sharded_pack_split(const State& s) { return s.sharded && s.comm != nullptr && !s.single_stream; }
// side_sync words: GammaV, the delta chains, Gamma2's prep (1 + nr), then the sharded Eta solve's
// all-reduce-B flag (sweep_sharded's edge-free sweeps)
constexpr int SIDE_ARB_SLOT = 2 + HMSC_MAX_LEVELS, SIDE_SYNC_INTS = SIDE_ARB_SLOT + 1;
inline int* arb_flag_ptr(State& s) { return s.side_sync + SIDE_ARB_SLOT; }
void launch_lambda_priors(State& s, uint32_t iter, hipStream_t st);
void launch_eta(State& s, uint32_t iter);
void launch_inv_sigma(State& s, uint32_t iter);
// record pack; slot == nullptr: device-chosen (graph replay).  part: 0 all, 1 the main-stream
// quantities (BL, Psi, iSigma, Eta), 2 the side-stream ones (Gamma, iV, Delta) on `side`
void launch_record(State& s, double* slot, int part = 0);
void launch_rec_copy(State& s, int k, int parts);
bool side_fusion_ok(const State& s);
// phylogeny branch (phylo.hip)
size_t phylo_work_doubles(int ns, int Kmax, int nc, int nrho);
void launch_phylo_gv_sums(State& s, uint32_t iter, hipStream_t st);
void launch_rho(State& s, uint32_t iter, hipStream_t st);
void launch_beta_lambda_phylo(State& s, uint32_t iter);
void launch_side_fused(State& s, uint32_t iter);
// blocked dense fp64 factorisation / solves (dense.hip)
// The dense handshake block (one per chain, State::trsv_sync, zero-initialised): [0] ticket,
// [1] done count, [2 + b] flag of 64-block b of a sync-free solve, [DENSE_SYNC_ERR] the error
// word every bounded in-launch wait raises a bit of on timeout (HS_ERR_*; the host checks it
// after a run, capi.cpp check_device_flags), [DENSE_SYNC_TEST] a test hook
// (hmsc_debug_poison).
constexpr int TRSV_SF_MAXB = 4096;
constexpr int DENSE_SYNC_ERR = 2 + TRSV_SF_MAXB;
constexpr int DENSE_SYNC_TEST = DENSE_SYNC_ERR + 1;
constexpr int DENSE_SYNC_INTS = DENSE_SYNC_ERR + 2;
enum HsErr { HS_ERR_TRSV_FLAG = 1, HS_ERR_TRSV_TICKET = 2, HS_ERR_CHOL_PANEL = 4 };
constexpr int HS_TEST_SKIP_PUBLISH = 1;  // DENSE_SYNC_TEST: the next fused panel step withholds its flag
// bw > 0: A is banded (A[i, j] = 0 for i - j > bw, entries outside the band zero on entry);
// the factor keeps the band, and only the band's tiles are touched (n bw^2 work instead of n^3).
// sync: the dense handshake block (enables the fused panel step), or null.
void dense_potrf_lower(hipStream_t st, double* A, int n, int lda, double* ws, int* info, int bw = 0,
                       int* sync = nullptr);
// sync: the dense handshake block for the one-launch sync-free solve, or null for one launch
// per 64-block
void dense_trsv_lower(hipStream_t st, const double* L, int n, int lda, double* x, int trans, double* ws, int bw = 0,
                      int* sync = nullptr);
void dense_trtri_lower(hipStream_t st, const double* L, int ldl, int n, double* M, int ldm, double* dinv,
                       bool have_dinv);
// workspace of dense_potrf_lower + dense_trsv_lower: the 64 x 64 diagonal-block inverses, then n
inline size_t dense_ws_doubles(int n) { return (size_t)((n + 63) / 64) * 64 * 64 + (size_t)n + 64; }
// rows per 64-column panel of the tile-band layout of a band matrix of bandwidth bw (pass
// lda = -dense_band_ld(bw) to dense_potrf_lower / dense_trsv_lower; dense.hip aix): the panel's
// diagonal tile, the tiles below it in the band, and one more for the transposed solve's
// tile-aligned reach
inline int dense_band_ld(int bw) { return 64 * (2 + (bw + 63) / 64); }
void dense_lauum_lower(hipStream_t st, const double* M, int ldm, int n, double* out, int ldo);
// out = U diag(d) U^T (full symmetric), d = dbase + n (*rho - 1) or its reciprocal
void dense_gram_diag(hipStream_t st, const double* U, int ldu, int n, const double* dbase, const double* rho,
                     bool recip, double* out, int ldo);
// the 'Full' alphapw grid on the device (R/computeDataParameters.R:53-81) from coordinates
// (np x sdim, column-major) or a distance matrix (np x np): RiWg = chol(W_g)^-1 (lower),
// iWg = RiWg^T RiWg, detWg = log det W_g
void spatial_full_grid(hipStream_t st, int np, int sdim, const double* coords, const double* dist,
                       const double* alphas, int G, double* iWg, double* RiWg, double* detWg, int* info);
// spatial "Full" levels (spatial.hip)
size_t spatial_work_doubles(const State& s, int r);
// NNGP level setup on the host: nearest earlier neighbours, Vecchia coefficients over the
// alphapw grid, detWg, the RCM factorization order and its bandwidth (device arrays of Level)
void setup_nngp_level(State& s, int r, const double* coords, int sdim, int k, const double* alphapw, int G);
void launch_eta_spatial(State& s, int r, uint32_t iter);
void launch_alpha(State& s, uint32_t iter);
// updateGammaEta (gamma_eta.hip)
size_t gamma_eta_work_doubles(const State& s);
void launch_gamma_eta(State& s, uint32_t iter);  // GammaV + LambdaPriors + Eta, co-launched
void join_side(State& s);
// a fresh zeroed device buffer of n doubles replacing `old` (freed), under the allocation
// lock every chain's captures respect (capi.cpp)
double* device_realloc_doubles(State& s, double* old, size_t n);
void launch_copied_flag(State& s, uint64_t value);
size_t record_slot_doubles(const State& s);
// ---- species-sharded sweep (kernels.hip); ar_point is the transport (capi.cpp)
struct ArbLayout {
  size_t zl = 0, cr = 0, gv = 0, rs = 0, na = 0, n = 0;  // offsets into ar_b, n = doubles in use
  int ldcr = 0;
};
ArbLayout arb_layout(const State& s);
size_t arb_capacity(const State& s);
void ar_point(State& s, double* buf, size_t n);
void sweep_sharded(State& s, uint32_t iter);
void run_updater_sharded(State& s, uint32_t which, uint32_t iter);
bool sharded_fused_ok(const State& s);
void read_stamps(double* out, int n);  // diagnostic build (HMSC_STAMPS)

}  // namespace hmsc
