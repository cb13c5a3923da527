// C ABI of hmsc_amd (include/hmsc_amd.h): chain state lifecycle, the sweep driver in
// the reference block order (R/sampleMcmc.R:219-306), recording, updateNf, RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <ucontext.h>

#include <algorithm>
#include <cmath>
#include <csignal>
#include <cstdio>
#include <atomic>
#include <cstring>
#include <cstdlib>
#include <thread>
#include <map>
#include <memory>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hmsc_amd.h"
#include "common.h"
#include "rng.h"
#include "state.h"

struct hmsc_state {
  hmsc::State s;
};

// ---------------------------- fault diagnostics ----------------------------
// HMSC_SEGV_DIAG=1: on SIGSEGV / SIGBUS print the faulting address and PC, every frame with
// the shared object (and symbol) it lies in, and the /proc/self/maps entries near the
// faulting address, then re-raise.  Stripped runtimes print as "(unknown)" in glog's handler
// (which rocprofv3 installs); this one names the library of each frame.  Diagnostic only.
namespace {
void fault_diag(int sig, siginfo_t* si, void* ctx) {
  const ucontext_t* uc = static_cast<const ucontext_t*>(ctx);
  void* pc = uc ? (void*)uc->uc_mcontext.gregs[REG_RIP] : nullptr;
  std::fprintf(stderr, "[hmsc] signal %d: fault address %p, pc %p\n", sig, si ? si->si_addr : nullptr, pc);
  void* fr[64];
  const int n = backtrace(fr, 64);
  for (int i = -1; i < n; ++i) {
    void* a = i < 0 ? pc : fr[i];
    Dl_info d{};
    if (a && dladdr(a, &d) && d.dli_fname)
      std::fprintf(stderr, "[hmsc]   #%d %p %s+0x%lx %s+0x%lx\n", i, a, d.dli_fname,
                   (unsigned long)((char*)a - (char*)d.dli_fbase), d.dli_sname ? d.dli_sname : "?",
                   d.dli_saddr ? (unsigned long)((char*)a - (char*)d.dli_saddr) : 0ul);
    else
      std::fprintf(stderr, "[hmsc]   #%d %p ?\n", i, a);
  }
  if (FILE* f = std::fopen("/proc/self/maps", "r")) {
    const uintptr_t fa = si ? (uintptr_t)si->si_addr : 0;
    char line[512];
    while (std::fgets(line, sizeof(line), f)) {
      unsigned long lo = 0, hi = 0;
      if (std::sscanf(line, "%lx-%lx", &lo, &hi) == 2 && hi + (64ul << 20) >= fa && lo <= fa + (64ul << 20))
        std::fprintf(stderr, "[hmsc]   map %s", line);
    }
    std::fclose(f);
  }
  std::fflush(stderr);
  std::signal(sig, SIG_DFL);
  std::raise(sig);
}
struct FaultDiagInstaller {
  FaultDiagInstaller() {
    const char* e = std::getenv("HMSC_SEGV_DIAG");
    if (!e || e[0] != '1') return;
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = fault_diag;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
    sigaction(SIGBUS, &sa, nullptr);
  }
} g_fault_diag;
}  // namespace

namespace hmsc {

static thread_local std::string g_last_error;
// live chains per device in this process (build_state / free_state, under g_dev_mu)
static std::map<int, int> g_live_chains;
// Chains may live on concurrent host threads (sampleMcmc nParallel, one stream each).  A
// stream capture must not overlap another thread's device-wide synchronising calls
// (hipMalloc / hipFree / hipDeviceSynchronize): those would invalidate it.  Captures,
// chain construction / destruction and every other allocation take this lock.
static std::recursive_mutex g_dev_mu;
// recorded samples in flight between device and host: two replays' worth (a replay's samples
// are copied and unpacked while the next replay runs), at most ~256 MB of pinned host memory
static constexpr int RING_SLOTS_MIN = 8;
static constexpr size_t RING_BYTES_MAX = (size_t)256 << 20;
// Kernel nodes per sweep graph.  rocprofv3 (rocprofiler-sdk, ROCm 7.2) fails inside its
// queue interception when a large graph is launched: SIGSEGV in librocprofiler-sdk.so called
// from hipGraphLaunch (config 3: 431-node one-sweep and 3448-node eight-sweep graphs,
// gpurun_out/s4_phy.err with HMSC_SEGV_DIAG=1), a hang for config 4's 512-node 64-sweep graph
// (s5_g64.err), while 256 / 288-node graphs (config 4 at 32 sweeps per graph) and the same
// phylo run without graphs (HMSC_NO_GRAPH=1) profile cleanly, and none of these graphs fail
// without the profiler.  Node count is not the whole story: after round 3's one-launch
// triangular solves config 3's one-sweep graph has 235 nodes and still faults under the
// profiler (gpurun_out/r03_s28_phyprof.err), while config 4's 256-node graphs do not.  Under
// rocprofv3 (it exports ROCPROF_OUTPUT_PATH to the program) graphs are therefore kept to 128
// nodes and sweeps that need more run eagerly (config 3 then profiles cleanly); otherwise the
// cap only bounds instantiation cost.  HMSC_GRAPH_MAX_NODES overrides either.
static size_t graph_max_nodes() {
  static const size_t cap = [] {
    if (const char* e = std::getenv("HMSC_GRAPH_MAX_NODES"))
      if (e[0]) return (size_t)std::max(1L, std::atol(e));
    return std::getenv("ROCPROF_OUTPUT_PATH") ? (size_t)128 : (size_t)8192;
  }();
  return cap;
}

int z_log_table_doubles();           // zdraw.hip
void z_log_table_fill(double* t);

static int graph_level(int n) {  // floor(log2 n)
  int k = 0;
  while ((1 << (k + 1)) <= n) ++k;
  return k;
}

static int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

template <class F>
static int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const HmscError& e) {
    return fail(e.code, e.what());
  } catch (const std::exception& e) {
    return fail(-3, e.what());
  } catch (...) {
    return fail(-4, "unknown error");
  }
}

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int d) {
    HIP_OK(hipGetDevice(&prev));
    if (prev != d) HIP_OK(hipSetDevice(d));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// Owners for the scratch device buffers and streams of one-shot entry points
// (hmsc_dense_chol_solve, hmsc_spatial_full_grid): freed on every exit, including an
// HmscError thrown by HIP_OK half way (guarded() turns it into an error code).
struct DevBufs {
  std::vector<void*> p;
  template <class T>
  T* alloc(size_t n) {
    void* q = nullptr;
    HIP_OK(hipMalloc(&q, std::max<size_t>(1, n) * sizeof(T)));
    p.push_back(q);
    return static_cast<T*>(q);
  }
  ~DevBufs() {
    for (void* q : p) (void)hipFree(q);
  }
};
struct OwnedStream {
  hipStream_t s = nullptr;
  OwnedStream() { HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
  ~OwnedStream() {
    if (s) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
  }
};

// ---------------------------- host dense helpers ----------------------------
using Mat = std::vector<double>;  // column-major

static void host_chol(Mat& A, int n) {  // lower in place, upper zeroed
  for (int c = 0; c < n; ++c) {
    double d = A[c + n * c];
    for (int k = 0; k < c; ++k) d -= A[c + n * k] * A[c + n * k];
    HMSC_REQUIRE(d > 0.0, "matrix is not positive definite");
    d = std::sqrt(d);
    A[c + n * c] = d;
    for (int i = c + 1; i < n; ++i) {
      double v = A[i + n * c];
      for (int k = 0; k < c; ++k) v -= A[i + n * k] * A[c + n * k];
      A[i + n * c] = v / d;
    }
  }
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < j; ++i) A[i + n * j] = 0.0;
}

static Mat host_inv_spd(const Mat& A, int n) {
  Mat L = A;
  host_chol(L, n);
  Mat Li(n * n, 0.0);
  for (int c = 0; c < n; ++c)
    for (int i = c; i < n; ++i) {
      double s = (i == c) ? 1.0 : 0.0;
      for (int k = c; k < i; ++k) s -= L[i + n * k] * Li[k + n * c];
      Li[i + n * c] = s / L[i + n * i];
    }
  Mat R(n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = std::max(i, j); k < n; ++k) s += Li[k + n * i] * Li[k + n * j];
      R[i + n * j] = s;
    }
  return R;
}

static Mat host_mm(const Mat& A, const Mat& B, int m, int k, int n) {
  Mat C(m * n, 0.0);
  for (int j = 0; j < n; ++j)
    for (int q = 0; q < k; ++q) {
      const double b = B[q + k * j];
      for (int i = 0; i < m; ++i) C[i + m * j] += A[i + m * q] * b;
    }
  return C;
}

// ---------------------------- device memory ----------------------------
// Host <-> device copies and fills go through non-blocking streams, never the legacy null
// stream: a legacy-stream operation in one thread while another thread's chain is capturing
// its sweep graph fails with "operation would make the legacy stream depend on a capturing
// blocking stream" (several chains driven from host threads of one process).
static hipStream_t thread_stream() {
  thread_local std::map<int, hipStream_t> streams;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  hipStream_t& st = streams[dev];
  if (!st) HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  return st;
}
static void copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st = nullptr) {
  if (!st) st = thread_stream();
  HIP_OK(hipMemcpyAsync(dst, src, bytes, kind, st));
  HIP_OK(hipStreamSynchronize(st));
}

template <class T>
static T* dalloc(size_t n) {
  T* p = nullptr;
  if (n == 0) n = 1;
  HIP_OK(hipMalloc(&p, n * sizeof(T)));
  const hipStream_t st = thread_stream();
  HIP_OK(hipMemsetAsync(p, 0, n * sizeof(T), st));
  HIP_OK(hipStreamSynchronize(st));
  return p;
}

double* device_realloc_doubles(State& s, double* old, size_t n) {
  std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
  DeviceGuard dg(s.device);
  HIP_OK(hipStreamSynchronize(s.stream));
  if (old) HIP_OK(hipFree(old));
  return dalloc<double>(n);
}

template <class T>
static T* dupload(const T* h, size_t n) {
  T* p = dalloc<T>(n);
  if (h && n) copy_sync(p, h, n * sizeof(T), hipMemcpyHostToDevice);
  return p;
}

template <class T>
static void h2d(T* d, const T* h, size_t n, hipStream_t st) {
  if (n) HIP_OK(hipMemcpyAsync(d, h, n * sizeof(T), hipMemcpyHostToDevice, st));
}

template <class T>
static void d2h(T* h, const T* d, size_t n, hipStream_t st) {
  if (n) HIP_OK(hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, st));
}

// The all-reduce of a sharded chain (state.h "species-sharded chain"): buf[0 .. n) summed over
// the ranks in place, on the chain's stream.  RCCL: one ncclAllReduce (captured into the sweep
// graphs like any kernel).  Host transport: the sum goes through pinned host memory and the
// caller's callback; inside a graph capture the capture is split here into segments, which
// hmsc_run replays with the callback between them.  Every call is counted (hmsc_debug_get
// "ar_calls"): a steady sweep issues two (kernels.hip sweep_sharded).
void ar_point(State& s, double* buf, size_t n) {
  if (n == 0) return;
  HMSC_REQUIRE(s.sharded, "internal: all-reduce on an unsharded chain");
  if (s.capturing) {
    ++s.ar_in_capture;  // (executed, and counted, by the replays)
  } else {
    ++s.ar_calls;
    s.ar_doubles += n;
  }
  if (s.comm) {
    // one rank: the in-place sum is the identity.  RCCL's one-rank path still issued a copy on
    // the copy engine the record ring's D2H copies use, so the first sweep of each replay
    // waited behind the previous replay's record copy (~130 us per replay boundary in the r06
    // traces); it is not issued (still counted: the sweep's all-reduce points are unchanged)
    if (s.nranks == 1) return;
    const ncclResult_t r = ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, (ncclComm_t)s.comm, s.stream);
    HMSC_REQUIRE(r == ncclSuccess, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return;
  }
  HMSC_REQUIRE(n <= s.ar_host_doubles, "internal: all-reduce larger than its host staging buffer");
  // a segment boundary may not leave the side stream forked; outside a capture the join keeps
  // the two transports' stream order alike
  join_side(s);
  HIP_OK(hipMemcpyAsync(s.ar_host, buf, n * sizeof(double), hipMemcpyDeviceToHost, s.stream));
  if (s.capturing && s.cap_segs) {
    hipGraph_t g = nullptr;
    HIP_OK(hipStreamEndCapture(s.stream, &g));
    s.cap_segs->emplace_back(g, n);
    HIP_OK(hipStreamBeginCapture(s.stream, hipStreamCaptureModeThreadLocal));
  } else {
    HMSC_REQUIRE(!s.capturing, "internal: host-transport all-reduce inside a capture without segments");
    HIP_OK(hipStreamSynchronize(s.stream));
    HMSC_REQUIRE(s.host_allreduce(s.ar_host, (int64_t)n, s.host_allreduce_ctx) == 0, "host all-reduce callback failed");
  }
  HIP_OK(hipMemcpyAsync(buf, s.ar_host, n * sizeof(double), hipMemcpyHostToDevice, s.stream));
}

// ---------------------------- phylogeny ----------------------------
// computeDataParameters' rho grid (R/computeDataParameters.R:19-39) in spectral form: with
// C = U diag(d) U^T every Q_g = U diag(q_g) U^T (phylo.hip), so the device keeps U, the table
// 1 / q_g,i and log(rhopw[g,2]) - nc/2 logdet Q_g instead of nrho dense ns x ns matrices.
static void setup_phylo(State& s, const hmsc_model* m) {
  const int ns = s.ns, nt = s.nt, nc = s.nc;
  HMSC_REQUIRE(m->C_vectors != nullptr && m->C_values != nullptr,
               "phylogeny: pass the eigendecomposition of C (C_vectors, C_values)");
  HMSC_REQUIRE(m->nrho > 0 && m->rhopw != nullptr, "phylogeny: rhopw grid missing");
  HMSC_REQUIRE(!s.sharded, "phylogeny couples all species: species-sharded chains are not supported");
  // NA in Y: R's phylogeny branch factors kronecker(XEtaTXEta, diag(iSigma)) + P over the
  // imputed Z with no per-species masking (R/updateBetaLambda.R:124-146), so the device's
  // phylogeny system takes the full Gram and an unmasked XZ (zdraw.hip mask_na = 0)
  s.phylo = true;
  s.nrho = m->nrho;
  std::vector<double> winv((size_t)s.nrho * ns), rbase(s.nrho);
  for (int i = 0; i < ns; ++i) HMSC_REQUIRE(m->C_values[i] > 0.0, "phylogeny: C must be positive definite");
  for (int g = 0; g < s.nrho; ++g) {
    const double rho = m->rhopw[g], pw = m->rhopw[g + s.nrho];
    double ld = 0.0;
    for (int i = 0; i < ns; ++i) {
      const double d = m->C_values[i];
      const double q = rho >= 0.0 ? rho * d + (1.0 - rho) : (-rho) / d + (1.0 + rho);
      HMSC_REQUIRE(q > 0.0, "phylogeny: Q_g not positive definite");
      winv[(size_t)ns * g + i] = 1.0 / q;
      ld += std::log(q);
    }
    rbase[g] = std::log(pw) - 0.5 * nc * ld;  // R/updateRho.R:19-20
  }
  std::vector<double> tt((size_t)ns * nt, 0.0);  // U^T Tr
  for (int q = 0; q < nt; ++q)
    for (int i = 0; i < ns; ++i) {
      double v = 0.0;
      for (int j = 0; j < ns; ++j) v += m->C_vectors[j + (size_t)ns * i] * m->Tr[j + (size_t)ns * q];
      tt[i + (size_t)ns * q] = v;
    }
  s.phU = dupload(m->C_vectors, (size_t)ns * ns);
  s.phWinv = dupload(winv.data(), winv.size());
  s.phRbase = dupload(rbase.data(), rbase.size());
  s.phTt = dupload(tt.data(), tt.size());
  s.phBt = dalloc<double>((size_t)nc * ns + 1);
  s.phEt = dalloc<double>((size_t)nc * ns + 1);
  s.phTTw = dalloc<double>((size_t)nt * nt);
  s.phNmax = s.Kmax * ns;
  HMSC_REQUIRE(s.phNmax <= 65536, "phylogeny: (nc + nfMax) * ns must be <= 65536 for the dense BetaLambda branch "
                                   "(a 34 GB system)");
  s.phWork = dalloc<double>(phylo_work_doubles(ns, s.Kmax, nc, s.nrho));
  s.mask &= ~(uint32_t)HMSC_UP_GAMMA2;  // updateGamma2 returns Gamma unchanged when C is given (R/updateGamma2.R:35-36)
}

// ---------------------------- create ----------------------------
// Species shard of `rank`: whole species quads (updateZ draws species 4q .. 4q + 3 from one
// Philox block), the ceil(ns / 4) quads spread as evenly as possible over the ranks: rank r owns
// quads [floor(r Q / n), floor((r + 1) Q / n)).  Every rank gets a quad when Q >= n; returns -1
// if this rank's shard is empty.
static int shard_range(int ns, int rank, int nranks, int* sp0, int* nsl) {
  const long quads = (ns + 3) / 4;
  const long q0 = quads * rank / nranks, q1 = quads * (rank + 1) / nranks;
  *sp0 = (int)std::min<long>(ns, 4 * q0);
  *nsl = (int)std::min<long>(ns, 4 * q1) - *sp0;
  return *nsl > 0 ? 0 : -1;
}

static int live_chains(int device) {
  std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
  auto it = g_live_chains.find(device);
  return it == g_live_chains.end() ? 0 : it->second;
}
int live_chains_on(int device) { return live_chains(device); }

static void build_state(State& s, const hmsc_model* m, uint64_t seed, int device, uint32_t mask, int rank,
                        int nranks, const void* comm_id, hmsc_allreduce_fn host_fn = nullptr,
                        void* host_ctx = nullptr) {
  std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
  // the device first: free_state decrements the count of s.device, whichever check below throws
  s.device = device;
  if (++g_live_chains[device] == 2) {
    // edge-free graphs (device-side joins) are only safe with one chain on a device: replays
    // launch under g_dev_mu after rechecking the count (replay_sweeps), and the ones already
    // queued by the chain that was alone drain here before this chain can launch anything
    DeviceGuard dg0(device);
    HIP_OK(hipDeviceSynchronize());
  }
  s.counted_live = true;
  HMSC_REQUIRE(m != nullptr, "model is NULL");
  HMSC_REQUIRE(m->struct_size == (int32_t)sizeof(hmsc_model),
               "hmsc_model.struct_size must be sizeof(hmsc_model) of include/hmsc_amd.h (rebuild the caller "
               "against this header and zero-initialise the struct)");
  HMSC_REQUIRE(m->ny > 0 && m->ns > 0 && m->nc >= 0 && m->nt > 0, "bad dimensions");
  HMSC_REQUIRE(m->nr >= 0 && m->nr <= HMSC_MAX_LEVELS, "nr out of range");
  s.ny = m->ny;
  s.ns = m->ns;
  s.nc = m->nc;
  s.nt = m->nt;
  s.nr = m->nr;
  s.device = device;
  s.mask = mask;
  s.rank = rank;
  s.nranks = nranks;
  s.key = Key{(uint32_t)(seed & 0xFFFFFFFFu), (uint32_t)(seed >> 32)};
  s.f0 = m->f0;
  // species shards start at even species: updateZ draws the species pair (2m, 2m+1) from one
  // Philox call (kernels.hip, z_wave_kernel)
  HMSC_REQUIRE(shard_range(m->ns, rank, nranks, &s.sp0, &s.nsl) == 0,
               "species shard is empty: a sharded chain needs at least 2 species per rank (shards start at even species)");
  DeviceGuard dg(device);
  HIP_OK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&s.copy_stream, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&s.side, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&s.side2, hipStreamNonBlocking));
  HIP_OK(hipEventCreateWithFlags(&s.ev_bl, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&s.ev_side, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&s.ev_side2, hipEventDisableTiming));
  s.host_allreduce = host_fn;
  s.host_allreduce_ctx = host_ctx;
  // sharded: more than one rank, or one rank given a communicator / host transport (the sharded
  // kernels and collectives on a single GPU: tests/test_gpu_sharded.py)
  s.sharded = nranks > 1 || comm_id != nullptr || host_fn != nullptr;
  if (s.sharded && host_fn == nullptr) {
    HMSC_REQUIRE(comm_id != nullptr, "sharded chain needs an RCCL unique id");
    ncclUniqueId id;
    std::memcpy(&id, comm_id, sizeof(id));
    ncclComm_t comm;
    const ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
    HMSC_REQUIRE(r == ncclSuccess, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    s.comm = comm;
  }
  const int ny = s.ny, nc = s.nc, nt = s.nt, nsl = s.nsl, sp0 = s.sp0, N = nc * nt;
  // levels
  int sum_nfmax = 0;
  for (int r = 0; r < s.nr; ++r) {
    Level& L = s.lev[r];
    L.spatial = m->sDim != nullptr && m->sDim[r] != 0;
    if (L.spatial) {
      HMSC_REQUIRE(m->spatialMethod != nullptr && m->spatialMethod[r] >= 1 && m->spatialMethod[r] <= 3,
                   "spatial level: spatialMethod must be 1 (Full), 2 (NNGP) or 3 (GPP)");
      HMSC_REQUIRE(m->spatialMethod[r] == 1 || m->np[r] == ny,
                   "spatial level: NNGP / GPP levels need np == ny (R/updateEta.R:140,165)");
      HMSC_REQUIRE(m->spatialMethod[r] != 2 || (m->sCoord[r] && m->nNeighbours),
                   "NNGP level: pass the unit coordinates (sCoord) and nNeighbours; nearest neighbours are not "
                   "available for distance matrices (R/computeDataParameters.R:86-88)");
      const bool geom = (m->spatialMethod[r] == 1 && !m->iWg[r] && (m->sCoord[r] || m->distMat[r])) ||
                        m->spatialMethod[r] == 2;
      const bool gpp = m->spatialMethod[r] == 3 && !m->iWg[r] && m->nKnots && m->nKnots[r] > 0 && m->idDg[r] &&
                       m->idDW12g[r] && m->Fg[r] && m->iFg[r] && m->detDg[r];
      HMSC_REQUIRE(m->nalpha == nullptr || m->nalpha[r] <= HMSC_MAX_ALPHA,
                   "spatial level: the alphapw grid may have at most 2048 rows in this build");
      HMSC_REQUIRE(m->nalpha != nullptr && m->nalpha[r] > 0 && m->alphapw[r] &&
                       (geom || gpp || (m->iWg[r] && m->RiWg[r] && m->detWg[r])),
                   "spatial level: alphapw and either iWg / RiWg / detWg (computeDataParameters' rLPar), "
                   "for 'Full' sCoord / distMat, or for 'GPP' nKnots / idDg / idDW12g / Fg / iFg / detDg must be given");
      HMSC_REQUIRE(!(mask & HMSC_UP_GAMMAETA) || m->spatialMethod[r] == 1,
                   "updataGammaEta: no method implemented yet for NNGP / GPP with GammaEta updater "
                   "(R/updateGammaEta.R:153-158): pass updater GammaEta=FALSE");
    }
    HMSC_REQUIRE(m->xDim == nullptr || m->xDim[r] == 0,
                 "a covariate-dependent level is passed as xDim consecutive levels sharing Eta "
                 "(hmsc_model etaShare / xScale), with xDim = 0 for each");
    {  // covariate-dependent level groups (etaShare / xScale, include/hmsc_amd.h)
      const int owner = (m->etaShare && m->etaShare[r] >= 0) ? m->etaShare[r] : r;
      HMSC_REQUIRE(owner <= r, "etaShare[r] must name r itself or an earlier level");
      if (owner < r) {
        HMSC_REQUIRE(s.lev[owner].eta_owner < 0 && owner + s.lev[owner].xgroup == r,
                     "etaShare: the levels sharing one Eta must be consecutive, after the level named");
        HMSC_REQUIRE(m->np[r] == m->np[owner] && m->nfMin[r] == m->nfMin[owner] && m->nfMax[r] == m->nfMax[owner],
                     "etaShare: levels sharing Eta need the same units and nfMin / nfMax");
        for (int i = 0; i < ny; ++i)
          HMSC_REQUIRE(m->Pi[i + (size_t)ny * r] == m->Pi[i + (size_t)ny * owner], "etaShare: levels sharing Eta need the same Pi");
        L.eta_owner = owner;
        s.lev[owner].xgroup++;
      }
      if (m->xScale[r] || owner < r) {
        HMSC_REQUIRE(m->xScale[r] != nullptr, "etaShare: every level of a shared-Eta group needs its xScale column");
        s.any_xs = true;
      }
    }
    HMSC_REQUIRE(!((m->xScale[r] != nullptr) && (L.spatial || s.sharded || (mask & HMSC_UP_GAMMAETA))),
                 "covariate-dependent levels: not with spatial levels, species sharding or updateGammaEta "
                 "(R/updateGammaEta.R and the spatial branches of R/updateEta.R take Lambda as a matrix): "
                 "pass updater GammaEta=FALSE");
    HMSC_REQUIRE(!(s.sharded && L.spatial), "spatial levels couple the units of every species' factors densely: "
                                            "species-sharded chains are not supported (run one chain per GPU)");
    L.np = m->np[r];
    L.nfmin = m->nfMin[r];
    L.nfmax = m->nfMax[r];
    L.nf = L.nfmin;
    L.nu = m->nu[r];
    L.a1 = m->a1[r];
    L.b1 = m->b1[r];
    L.a2 = m->a2[r];
    L.b2 = m->b2[r];
    sum_nfmax += L.nfmax;
  }
  // K = nc + sum(nf) <= HMSC_KCAP (128) is this build's kernel limit (16-row MFMA blocks of
  // updateZ, NKB <= 8; K x K factors in LDS).  R's default nfMax = Inf becomes ns
  // (R/Hmsc.R:554), so a default model with many species may ask for more factors than the
  // device holds: every level's buffers and record slots then hold nfcap = min(nfMax, 128 - nc
  // - the other levels' nfMin) factors (hmsc_get_nf_cap; the Python wrapper warns, or refuses
  // with nf_capacity="error"), and the chain stops with an explicit error only if updateNf
  // actually has to grow a level past it (MGP shrinkage keeps the adapted nf far below that in
  // practice).  The capacity beyond every level's nfMin is shared: a level may be refused below
  // its nfcap when the other levels have already grown into it (K would pass Kmax).
  HMSC_REQUIRE(nc + [&] { int v = 0; for (int r = 0; r < s.nr; ++r) v += s.lev[r].nfmin; return v; }() <= HMSC_KCAP,
               "nc + sum(nfMin) exceeds 128: this build's limit is K = nc + sum(nf) <= 128");
  s.Kmax = std::min(nc + sum_nfmax, HMSC_KCAP);
  s.NFmax = s.Kmax - nc;
  s.refresh_dims();
  for (int r = 0; r < s.nr; ++r) {
    Level& L = s.lev[r];
    int others = 0;
    for (int q = 0; q < s.nr; ++q)
      if (q != r) others += s.lev[q].nfmin;
    L.nfcap = std::max(L.nfmin, std::min(L.nfmax, s.NFmax - others));
    L.nf_alloc = std::max(1, L.nf);
    const int nfcap = L.nfcap;
    L.Eta = L.eta_alias() ? s.lev[L.eta_owner].Eta : dalloc<double>((size_t)L.np * nfcap);
    if (m->xScale[r]) L.xs = dupload(m->xScale[r], (size_t)L.np);
    std::vector<int> pi(ny), cnt(L.np + 1, 0), rows(ny);
    for (int i = 0; i < ny; ++i) {
      const int u = m->Pi[i + (size_t)ny * r] - 1;
      HMSC_REQUIRE(u >= 0 && u < L.np, "Pi out of range");
      pi[i] = u;
      cnt[u + 1]++;
    }
    for (int q = 0; q < L.np; ++q) cnt[q + 1] += cnt[q];
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (int i = 0; i < ny; ++i) rows[fill[pi[i]]++] = i;
    for (int q = 0; q < L.np; ++q) HMSC_REQUIRE(cnt[q + 1] > cnt[q], "a random-level unit has no rows");
    L.uniform_n = cnt[1] - cnt[0];
    for (int q = 0; q < L.np; ++q)
      if (cnt[q + 1] - cnt[q] != L.uniform_n) L.uniform_n = 0;
    L.Pi = dupload(pi.data(), ny);
    L.unit_ptr = dupload(cnt.data(), L.np + 1);
    L.unit_rows = dupload(rows.data(), ny);
    std::vector<int> alpha(std::max(1, L.nfcap), 1);
    L.Alpha = dupload(alpha.data(), alpha.size());
    std::vector<double> alphad(alpha.size(), 1.0);  // Alpha = rep(1, nf) (R/computeInitialParameters.R:216-221)
    L.AlphaD = dupload(alphad.data(), alphad.size());
    if (L.spatial) {
      const size_t G = m->nalpha[r], np2 = (size_t)L.np * L.np;
      L.nalpha = (int)G;
      L.alphapw = dupload(m->alphapw[r], 2 * G);
      if (m->spatialMethod[r] == 2) {  // NNGP in the sparse Vecchia form (spatial.hip)
        std::vector<double> alphas(m->alphapw[r], m->alphapw[r] + G);
        setup_nngp_level(s, r, m->sCoord[r], m->sDim[r], m->nNeighbours[r], alphas.data(), (int)G);
      } else if (m->spatialMethod[r] == 3 && !m->iWg[r]) {  // GPP in R's low-rank form
        const size_t nK = (size_t)m->nKnots[r];
        // gpp_alpha_kernel / launch_eta_gpp stage one knot vector in a 1024-entry LDS array
        // (spatial.hip); refuse larger knot sets here, before any updater can run
        HMSC_REQUIRE(nK <= 1024, "GPP level: at most 1024 knots in this build");
        L.gpp = true;
        L.nK = (int)nK;
        L.idDg = dupload(m->idDg[r], (size_t)L.np * G);
        L.idDW12g = dupload(m->idDW12g[r], (size_t)L.np * nK * G);
        L.Fg = dupload(m->Fg[r], nK * nK * G);
        L.iFg = dupload(m->iFg[r], nK * nK * G);
        L.detWg = dupload(m->detDg[r], G);
      } else if (m->iWg[r]) {
        L.iWg = dupload(m->iWg[r], np2 * G);
        L.RiWg = dupload(m->RiWg[r], np2 * G);
        L.riw_lower = m->spatialMethod[r] == 2 || m->spatialMethod[r] == 3;
        L.detWg = dupload(m->detWg[r], G);
      } else {  // 'Full' grid from the level's geometry, on the device
        L.iWg = dalloc<double>(np2 * G);
        L.RiWg = dalloc<double>(np2 * G);
        L.detWg = dalloc<double>(G);
        L.riw_lower = 1;
        const bool crd = m->sCoord[r] != nullptr;
        HMSC_REQUIRE(!crd || m->sDim[r] > 0, "spatial level: sDim must give the coordinate columns");
        int* flag = dalloc<int>(1);
        double* geo = crd ? dupload(m->sCoord[r], (size_t)L.np * m->sDim[r]) : dupload(m->distMat[r], np2);
        std::vector<double> alphas(m->alphapw[r], m->alphapw[r] + G);
        spatial_full_grid(s.stream, L.np, crd ? m->sDim[r] : 0, crd ? geo : nullptr, crd ? nullptr : geo,
                          alphas.data(), (int)G, L.iWg, L.RiWg, L.detWg, flag);
        HIP_OK(hipStreamSynchronize(s.stream));
        HIP_OK(hipFree(geo));
        int bad = 0;
        copy_sync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost);
        HIP_OK(hipFree(flag));
        HMSC_REQUIRE(bad == 0, "spatial level: a grid matrix W_g = exp(-d / alpha_g) is not positive definite "
                               "(duplicated coordinates?)");
      }
      {  // the spatial workspace (NNGP: the band in its tile-band layout, np nf x (bw + 128)):
         // a clear create-time error instead of an allocation failure mid-setup
        const size_t need = spatial_work_doubles(s, r) * sizeof(double);
        size_t free_b = 0, total_b = 0;
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        HMSC_REQUIRE(need < free_b, "spatial level " + std::to_string(r) + ": its workspace needs " +
                                        std::to_string(need >> 20) + " MiB (the " +
                                        (L.nngp ? std::string("NNGP band matrix, np nf x (bw + 128)") :
                                                  std::string("(np nf)^2 dense system")) +
                                        "), " + std::to_string(free_b >> 20) + " MiB free on the device");
      }
      L.spWork = dalloc<double>(spatial_work_doubles(s, r));
    }
  }
  // local species slices
  std::vector<int8_t> ycode((size_t)ny * nsl);
  std::vector<double> yval((size_t)ny * nsl), yraw((size_t)ny * nsl), trl((size_t)nsl * nt);
  std::vector<int> fam(nsl), var(nsl);
  std::vector<double> as(nsl), bs(nsl);
  std::vector<int> na_cols, na_index(nsl, -1);
  // rows with any NA in the WHOLE Y (every rank of a sharded chain must agree on them: updateEta's
  // NA rows, R/updateEta.R:59-70); NA in this rank's own species: has_na
  std::vector<int8_t> row_na(ny, 0);
  for (int jg = 0; jg < m->ns; ++jg)
    for (int i = 0; i < ny; ++i)
      if (std::isnan(m->Y[i + (size_t)ny * jg])) row_na[i] = 1, s.any_na_global = true;
  for (int j = 0; j < nsl; ++j) {
    const int jg = sp0 + j;
    fam[j] = m->distr[jg];
    var[j] = m->distr[jg + (size_t)m->ns];
    HMSC_REQUIRE(fam[j] >= 1 && fam[j] <= 3, "distr family must be 1 (normal), 2 (probit) or 3 (Poisson)");
    if (fam[j] != 2) s.all_probit = false;
    if (fam[j] == 1) s.any_normal = true;
    if (fam[j] == 3) s.any_poisson = true;
    if (var[j] == 1) s.any_var = true;
    as[j] = m->aSigma[jg];
    bs[j] = m->bSigma[jg];
    for (int q = 0; q < nt; ++q) trl[j + (size_t)nsl * q] = m->Tr[jg + (size_t)m->ns * q];
    bool col_na = false;
    for (int i = 0; i < ny; ++i) {
      const double y = m->Y[i + (size_t)ny * jg];
      const size_t c = i + (size_t)ny * j;
      yval[c] = y;
      yraw[c] = m->Yraw ? m->Yraw[i + (size_t)ny * jg] : y;
      if (std::isnan(y)) {
        ycode[c] = -1;
        col_na = true;
      } else {
        ycode[c] = (fam[j] == 2 && y != 0.0) ? 1 : 0;
      }
    }
    if (col_na) {
      na_index[j] = (int)na_cols.size();
      na_cols.push_back(j);
    }
  }
  s.has_na = !na_cols.empty();
  ycode.resize((size_t)ny * (nsl + 32) + 64, 0);  // z kernel loads past the last species (z_kernel.h ZArgs)
  s.Ycode = dupload(ycode.data(), ycode.size());
  {  // the z kernel's packed codes: word (species block b, site i) holds code + 1 of species
     // 32 b + jj in bits 2 jj, 2 jj + 1 (padding: code 0)
    const int nblk = (nsl + 31) / 32;
    std::vector<uint64_t> yb((size_t)nblk * ny + 64, 0x5555555555555555ull);
    for (int j = 0; j < nsl; ++j) {
      const int sh = 2 * (j % 32);
      for (int i = 0; i < ny; ++i) {
        uint64_t& w = yb[(size_t)(j / 32) * ny + i];
        w = (w & ~(3ull << sh)) | ((uint64_t)(ycode[i + (size_t)ny * j] + 1) << sh);
      }
    }
    s.Ybits = dupload(yb.data(), yb.size());
  }
  {  // the z kernel's log table (z_kernel.h log_tab)
    std::vector<double> lt(z_log_table_doubles());
    z_log_table_fill(lt.data());
    s.logtab = dupload(lt.data(), lt.size());
  }
  if (!s.all_probit) {
    s.Yval = dupload(yval.data(), yval.size());
    s.Yraw = dupload(yraw.data(), yraw.size());
  }
  s.fam = dupload(fam.data(), nsl);
  s.varest = dupload(var.data(), nsl);
  s.aSigma = dupload(as.data(), nsl);
  s.bSigma = dupload(bs.data(), nsl);
  s.Tr = dupload(trl.data(), trl.size());
  s.X = dupload(m->X, (size_t)ny * nc);
  s.n_na_cols = (int)na_cols.size();
  s.h_na_cols = na_cols;
  if (s.has_na) {
    s.na_cols = dupload(na_cols.data(), na_cols.size());
    s.na_index = dupload(na_index.data(), nsl);
    s.Gna = dalloc<double>((size_t)s.n_na_cols * s.Kmax * s.Kmax);
  }
  if (s.any_na_global) {
    std::vector<int> na_rows, slot(ny, -1);
    for (int i = 0; i < ny; ++i)
      if (row_na[i]) {
        slot[i] = (int)na_rows.size();
        na_rows.push_back(i);
      }
    s.n_na_rows = (int)na_rows.size();
    s.na_rows = dupload(na_rows.data(), na_rows.size());
    s.row_na = dupload(row_na.data(), ny);
    s.row_slot = dupload(slot.data(), ny);
    s.Msmall = dalloc<double>((size_t)s.n_na_rows * (s.NFmax * s.NFmax + s.NFmax));
  }
  // priors and constants (host precompute)
  Mat X(m->X, m->X + (size_t)ny * nc), XX(nc * nc, 0.0), TT(nt * nt, 0.0);
  for (int a = 0; a < nc; ++a)
    for (int b = 0; b < nc; ++b) {
      double v = 0.0;
      for (int i = 0; i < ny; ++i) v += X[i + (size_t)ny * a] * X[i + (size_t)ny * b];
      XX[a + nc * b] = v;
    }
  for (int a = 0; a < nt; ++a)
    for (int b = 0; b < nt; ++b) {
      double v = 0.0;
      for (int j = 0; j < m->ns; ++j) v += m->Tr[j + (size_t)m->ns * a] * m->Tr[j + (size_t)m->ns * b];
      TT[a + nt * b] = v;
    }
  Mat UG(m->UGamma, m->UGamma + (size_t)N * N);
  Mat iUG = host_inv_spd(UG, N);
  Mat UGL = UG;
  host_chol(UGL, N);
  Mat iV0(nc * nc);
  for (int a = 0; a < nc; ++a)
    for (int b = 0; b < nc; ++b) iV0[a + nc * b] = iUG[a + N * b];  // iUGamma[1:nc,1:nc] (R/updateGamma2.R:37)
  Mat V0g = host_inv_spd(iV0, nc);
  Mat V0gXX = host_mm(V0g, XX, nc, nc, nc);
  Mat V0gXXV0g = host_mm(V0gXX, V0g, nc, nc, nc);
  Mat V0(m->V0, m->V0 + (size_t)nc * nc);
  Mat V0inv = host_inv_spd(V0, nc);
  s.XX = dupload(XX.data(), XX.size());
  s.TT = dupload(TT.data(), TT.size());
  s.iUGamma = dupload(iUG.data(), iUG.size());
  s.UGammaL = dupload(UGL.data(), UGL.size());
  s.UGamma = dupload(UG.data(), UG.size());
  s.iV0 = dupload(iV0.data(), iV0.size());
  s.V0g = dupload(V0g.data(), V0g.size());
  s.V0gXXV0g = dupload(V0gXXV0g.data(), V0gXXV0g.size());
  s.V0gXX = dupload(V0gXX.data(), V0gXX.size());
  s.g2prep = dalloc<double>(2 * (size_t)nc * nc + 2 * (size_t)N * N);
  s.V0 = dupload(V0.data(), V0.size());
  s.V0inv = dupload(V0inv.data(), V0inv.size());
  s.mGamma = dupload(m->mGamma, (size_t)N);
  Mat iUmG(N, 0.0);
  for (int a = 0; a < N; ++a)
    for (int b = 0; b < N; ++b) iUmG[a] += iUG[a + N * b] * m->mGamma[b];
  s.iUmG = dupload(iUmG.data(), N);
  // state
  s.Z = dalloc<double>((size_t)ny * nsl);
  s.BL = dalloc<double>((size_t)s.Kmax * nsl);
  s.Psi = dalloc<double>((size_t)std::max(1, s.NFmax) * nsl);
  s.Delta = dalloc<double>(std::max(1, s.NFmax));
  s.Gamma = dalloc<double>(N);
  s.iV = dalloc<double>((size_t)nc * nc);
  s.iSigma = dalloc<double>(nsl);
  s.rho = dalloc<double>(1);
  {
    const double one = 1.0;  // rho = 1 (R/computeInitialParameters.R:226)
    copy_sync(s.rho, &one, sizeof(double), hipMemcpyHostToDevice, s.stream);
  }
  if (m->C != nullptr) setup_phylo(s, m);
  // workspaces
  const int n_tiles = (ny + 63) / 64;
  s.ntile_j = (nsl + 31) / 32;
  // four rounds of the resident z workgroups: a grid of exactly one round leaves every
  // workgroup displaced by a concurrent side-stream kernel to run after the round (measured
  // 142 us vs 104 us per launch at the config-4 size, scripts/z_chunk_sweep.sh); 16 / 24 / 32 /
  // 48 / 64 / 96 chunks at config 4: z 90 / 91 / 82 / 83 / 79 / 80 us (round 5, HMSC_Z_CHUNKS)
  s.nchunk = std::max(1, std::min(n_tiles, 4 * z_resident_slots(s) / std::max(1, s.ntile_j)));
  if (const char* e = std::getenv("HMSC_Z_CHUNKS"))  // tuning knob: site chunks of the z grid
    if (std::atoi(e) > 0) s.nchunk = std::max(1, std::min(n_tiles, std::atoi(e)));
  const int n_sblk = (ny + 63) / 64;
  s.zl_split = std::max(1, std::min(std::min(16, (nsl + 3) / 4), (640 + n_sblk - 1) / n_sblk));
  s.XZ = dalloc<double>((size_t)s.Kmax * nsl);
  s.XEta = dalloc<double>((size_t)ny * z_xeta_cols_for(s.Kmax) + 64);  // padded (z_kernel.h ZArgs)
  s.G = dalloc<double>((size_t)s.Kmax * s.Kmax);
  s.ZTr = dalloc<double>((size_t)ny * nt);
  s.XZ_part = dalloc<double>((size_t)s.nchunk * s.Kmax * nsl);
  s.bl_pre = dalloc<double>((size_t)64 * nsl);
  s.bl_pre_tag = dalloc<int>(2);
  HIP_OK(hipMemset(s.bl_pre_tag, 0xff, 2 * sizeof(int)));  // (sweep -1, K -1): nothing drawn yet
  s.G_part = dalloc<double>(std::max((size_t)std::max(std::max(s.nchunk, 64), (ny + 31) / 32) * s.Kmax * s.Kmax,
                                      (size_t)((ny + 15) / 16) * s.Kmax * std::max(1, s.NFmax)));
  s.ZTr_part = dalloc<double>((size_t)s.ntile_j * ny * nt);
  const int nfm = std::max(1, s.NFmax);
  s.ZL = dalloc<double>((size_t)ny * nfm);
  s.ZL_part = dalloc<double>((size_t)s.zl_split * ny * nfm);
  s.CR = dalloc<double>((size_t)s.Kmax * nfm);
  s.CR_part = dalloc<double>((size_t)((nsl + 31) / 32) * s.Kmax * nfm);
  s.LS = dalloc<double>((size_t)std::max(nfm, 16) * nsl);  // [species][16] (cr_body)
  s.etaW = dalloc<double>(16 * 16);
  {  // crw_kernel: 4 parts x 4 tiles x 16 x 16; bl_tail: (nbl + ngroups) tiles of CRW_TILE (520)
    const size_t nbl = (size_t)(nsl + 3) / 4, ngr = (nbl + 15) / 16;
    s.crw_part = dalloc<double>(std::max((size_t)4 * 4 * 256, (nbl + ngr) * 520));
    s.crw_ticket = dalloc<int>(3 + ngr);  // dalloc zero-fills
    s.crw_flag = s.crw_ticket + 2 + ngr;
    s.gvt_ld = nc * nc + N + nfm;             // [A nc^2 | BTr nc nt | rs NF]
    s.gvt = dalloc<double>((nbl + ngr) * (size_t)s.gvt_ld);
  }
  s.side_sync = dalloc<int>(SIDE_SYNC_INTS);
  s.Gamma_side = dalloc<double>(N);
  // under rocprofv3 (ROCPROF_OUTPUT_PATH, as for the graph node cap) the side chain keeps its
  // graph edges: counter passes serialise dispatches, and a device-side join would wait on a
  // launch queued behind it until its time bound (error -5); the kernel tracer delays the side
  // queue's dispatches enough that the traced durations would not be the sweep's
  if (std::getenv("ROCPROF_OUTPUT_PATH")) s.edge_free = false;
  if (const char* e = std::getenv("HMSC_SIDE_EDGES")) s.edge_free = e[0] != '1';
  if (const char* e = std::getenv("HMSC_SIDE_PARTIALS")) s.side_partials = e[0] == '1';
  if (const char* e = std::getenv("HMSC_LONG_TAIL")) s.long_tail = e[0] == '1';
  if (const char* e = std::getenv("HMSC_FIRST_REPLAY")) s.first_replay = std::max(0, atoi(e));
  // (GammaV's final stage and Gamma2's prep / final stage keep their N = nc nt systems here when
  // they do not fit a workgroup's LDS: 3 N^2 + 7 nc^2 doubles and the final stage's arrays)
  s.scratch_doubles = std::max<size_t>(1 << 20, 6 * (size_t)nc * nc + 2 * (size_t)N + (size_t)N * N);
  s.scratch = dalloc<double>(s.scratch_doubles);
  s.scratch2_doubles = std::max<size_t>(1 << 20, 7 * (size_t)nc * nc + 3 * (size_t)N * N + 16 + 8 * (size_t)N +
                                                     (size_t)nfm * nt + 2 * 1024 + 8 * 64 + 16);
  s.scratch2 = dalloc<double>(s.scratch2_doubles);
  s.psi_rs = dalloc<double>((size_t)64 * nfm);
  // (the species-block partials of GammaV (32 species a block) and Gamma2 (G2SB = 8))
  s.ABpart = dalloc<double>((size_t)((nsl + 7) / 8) * (nc * nc + 2 * N + nfm * nt + 8));
  s.allreduce_buf = dalloc<double>((size_t)nc * nc + 2 * N + nfm * nt + nfm + 64);
  if (s.sharded) {  // the two all-reduce buffers (state.h) and the host transport's staging
    const size_t na = (size_t)N + (size_t)nfm * nt + 8, nb = arb_capacity(s);
    s.ar_a = dalloc<double>(na);
    s.ar_b = dalloc<double>(nb);
    s.shard_ticket = dalloc<int>(4);
    if (s.host_allreduce) {
      s.ar_host_doubles = std::max(na, nb);
      HIP_OK(hipHostMalloc(&s.ar_host, sizeof(double) * s.ar_host_doubles, hipHostMallocDefault));
    }
  }
  // the device error / handshake words in one block (dalloc zero-fills), so the host reads
  // every error word with one copy: [dev_flags 16 | gbl_sync 4 | trsv_sync DENSE_SYNC_INTS]
  s.dev_flags = dalloc<int>(16 + 4 + DENSE_SYNC_INTS);
  s.gbl_sync = s.dev_flags + 16;
  s.trsv_sync = s.dev_flags + 20;
  s.d_iters = dalloc<uint32_t>(64);  // graph_sweeps <= 64
  s.d_iter = s.d_iters;
  if (s.mask & HMSC_UP_GAMMAETA) {  // updateGammaEta: dense (nc ns)^2 / joint spatial systems
    HMSC_REQUIRE(!s.sharded, "updateGammaEta cannot run on a species-sharded chain: pass updater GammaEta=FALSE");
    HMSC_REQUIRE((size_t)nc * s.ns <= 32768, "updateGammaEta: nc * ns must be <= 32768 (dense (nc ns)^2 systems, 4 x 8.6 GB)");
    // sized for the levels' nf now (nfMin); launch_gamma_eta grows it if updateNf adds factors
    for (int r = 0; r < s.nr; ++r)
      HMSC_REQUIRE(!s.lev[r].spatial || (size_t)nc * s.nt + (size_t)s.lev[r].np * s.lev[r].nf <= 32768,
                   "updateGammaEta, spatial level: nc nt + np nf must be <= 32768 (dense joint system, 8.6 GB)");
    s.geWork_doubles = gamma_eta_work_doubles(s);
    s.geWork = dalloc<double>(s.geWork_doubles);
  }
  {
    const char* g = getenv("HMSC_GRAPH_SWEEPS");
    // a power of two (remainders replay graphs of the smaller powers); one replay launch per
    // 32 sweeps at a steady state (8 was +1.8 % over 4)
    s.graph_sweeps = 1 << graph_level(g ? std::max(1, std::min(64, atoi(g))) : 32);
    // a host-transport sharded chain replays one sweep at a time (its all-reduces run on the
    // host between the segments of the sweep graph)
    if (s.sharded && s.comm == nullptr) s.graph_sweeps = 1;
  }
  // recording ring: device slots for two replays, their pinned host mirror and the copied
  // counter, allocated once here so no run pays for pinning
  s.slot_doubles = record_slot_doubles(s);
  {
    const size_t fit = RING_BYTES_MAX / std::max<size_t>(1, sizeof(double) * s.slot_doubles);
    s.ring_slots = (int)std::max<size_t>(RING_SLOTS_MIN, std::min<size_t>(2 * (size_t)s.graph_sweeps, fit));
    while (s.graph_sweeps > 1 && 2 * s.graph_sweeps > s.ring_slots) s.graph_sweeps >>= 1;
  }
  s.ring = dalloc<double>(s.slot_doubles * s.ring_slots);
  HIP_OK(hipHostMalloc(&s.host_rec, sizeof(double) * s.slot_doubles * s.ring_slots, hipHostMallocDefault));
  HIP_OK(hipHostMalloc(&s.copied_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_OK(hipHostGetDevicePointer((void**)&s.copied_dev, s.copied_host, 0));
  s.d_rec_desc = dalloc<int32_t>(8);  // {iter0, transient, thin, samples, run nonce}
  // kernel copies for the recorded graphs of at most kcopy_max sweeps: a run's first and last
  // replays, while long replays keep one host-issued copy each (HMSC_KERNEL_COPY=0: never,
  // HMSC_KERNEL_COPY_MAX: the size bound; a 32-sweep graph with kernel copies measured 2.9 %
  // slower over 1000 sweeps, the 20-step line 5 % faster, profiles/r06_kcopy_ab.txt).  With
  // them a run starts on a replay of at most 4 sweeps (HMSC_FIRST_REPLAY overrides): the device
  // starts after a short graph's submission instead of a 16- or 32-sweep one's, and a 20-sweep
  // run is 4 + 16 replays with kernel copies throughout (bound 16): the 20-step line ahead in
  // 10 of 12 same-box rounds (5,958 -> 6,210 over 7), 1000 steps unchanged
  // (profiles/r06_first_replay_ab.txt)
  {
    const char* e = std::getenv("HMSC_KERNEL_COPY");
    // (HMSC_SIDE_EDGES=1, the counter-collection profiler's serialised dispatches: a copy kernel
    // waiting on the device for a pack queued behind it would time out -- host copies then)
    s.kcopy = !(e && e[0] == '0') && s.edge_free;
    const char* m = std::getenv("HMSC_KERNEL_COPY_MAX");
    s.kcopy_max = m ? std::max(0, atoi(m)) : 16;
    if (!std::getenv("HMSC_FIRST_REPLAY")) s.first_replay = s.kcopy ? 4 : 0;
  }
  if (s.kcopy && hipHostGetDevicePointer((void**)&s.host_rec_dev, s.host_rec, 0) != hipSuccess) {
    (void)hipGetLastError();
    s.kcopy = false;  // (the host ring is not mapped for the device: host-issued copies)
  }
  s.pack_flags = dalloc<uint64_t>((size_t)3 * s.ring_slots);
  s.pack_ticket = dalloc<int>(4);
  s.d_iter_side = dalloc<uint32_t>(1);
  s.gv_part = dalloc<double>((size_t)((nsl + 31) / 32) * (nc * nc + nc * nt));
  HIP_OK(hipEventCreateWithFlags(&s.ev_graph, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&s.ev_ext, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&s.ev_ext_go, hipEventDisableTiming));
  s.d_ext_iter = dalloc<uint32_t>(64);
  {
    const char* g1 = getenv("HMSC_SINGLE_STREAM");
    s.single_stream = g1 && g1[0] == '1';
    const char* g = getenv("HMSC_NO_GRAPH");
    s.use_graph = !(g && g[0] && g[0] != '0');
  }
  HIP_OK(hipDeviceSynchronize());
}

static void free_state(State& s) {
  std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
  if (s.counted_live) --g_live_chains[s.device];
  s.counted_live = false;
  DeviceGuard dg(s.device);
  (void)hipDeviceSynchronize();
  s.unpack_pool.reset();  // idle between runs; joined before the host ring goes
  void* ptrs[] = {s.pack_flags, s.pack_ticket, s.X, s.Tr, s.Yval, s.Yraw, s.Ycode, s.Ybits, s.logtab, s.fam, s.varest, s.V0, s.iUGamma, s.mGamma, s.UGammaL,
                  s.aSigma, s.bSigma, s.XX, s.TT, s.V0g, s.V0gXXV0g, s.iV0, s.V0inv, s.iUmG, s.V0gXX, s.g2prep, s.scratch2, s.na_cols, s.na_index,
                  s.na_rows, s.row_na, s.row_slot, s.dev_flags, s.Z, s.XEta, s.BL, s.Psi, s.Delta, s.Gamma, s.iV,
                  s.iSigma, s.rho, s.XZ, s.G, s.ZTr, s.XZ_part, s.bl_pre, s.bl_pre_tag, s.G_part, s.ZTr_part, s.Gna, s.ZL, s.ZL_part,
                  s.CR, s.CR_part, s.LS, s.etaW, s.crw_part, s.crw_ticket, s.gvt, s.side_sync, s.Gamma_side, s.Msmall, s.scratch, s.psi_rs, s.ABpart, s.dbg_prec, s.ring, s.allreduce_buf,
                  s.phU, s.phWinv, s.phRbase, s.phTt, s.phBt, s.phEt, s.phTTw, s.phWork, s.UGamma, s.geWork};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (int r = 0; r < s.nr; ++r) {
    Level& L = s.lev[r];
    void* lp[] = {L.eta_alias() ? nullptr : L.Eta, L.xs, L.Pi, L.unit_ptr, L.unit_rows, L.Alpha, L.AlphaD, L.alphapw, L.iWg, L.RiWg, L.detWg, L.spWork,
                  L.idDg, L.idDW12g, L.Fg, L.iFg, L.nnIdx, L.nnA, L.nnD, L.nnPerm, L.nnPos, L.nnChPtr, L.nnCh};
    for (void* p : lp)
      if (p) (void)hipFree(p);
  }
  if (s.ev_graph) (void)hipEventDestroy(s.ev_graph);
  if (s.d_rec_desc) (void)hipFree(s.d_rec_desc);
  if (s.d_iter_side) (void)hipFree(s.d_iter_side);
  if (s.gv_part) (void)hipFree(s.gv_part);
  if (s.host_rec) (void)hipHostFree(s.host_rec);
  if (s.copied_host) (void)hipHostFree(s.copied_host);
  if (s.ar_host) (void)hipHostFree(s.ar_host);
  for (void* p : {(void*)s.ar_a, (void*)s.ar_b, (void*)s.shard_ticket})
    if (p) (void)hipFree(p);
  for (auto& v : s.gseg)
    for (auto& g : v)
      if (g.g) (void)hipGraphExecDestroy(g.g);
  for (auto& row : s.gx)
    for (hipGraphExec_t g : row)
      if (g) (void)hipGraphExecDestroy(g);
  if (s.d_iters) (void)hipFree(s.d_iters);
  if (s.d_kt) (void)hipFree(s.d_kt);
  if (s.comm) ncclCommDestroy((ncclComm_t)s.comm);
  if (s.ev_bl) (void)hipEventDestroy(s.ev_bl);
  if (s.ev_side) (void)hipEventDestroy(s.ev_side);
  if (s.ev_side2) (void)hipEventDestroy(s.ev_side2);
  if (s.ev_ext) (void)hipEventDestroy(s.ev_ext);
  if (s.ev_ext_go) (void)hipEventDestroy(s.ev_ext_go);
  if (s.side) (void)hipStreamDestroy(s.side);
  if (s.side2) (void)hipStreamDestroy(s.side2);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  if (s.copy_stream) (void)hipStreamDestroy(s.copy_stream);
}

// Wait on the main stream for the side-stream work of the previous sweep (it writes Gamma,
// iV, Psi, Delta and Gamma2's iV-only matrices).
// The main stream waits for everything enqueued on the side streams so far.
void join_side(State& s) {
  if (s.side_pending & 1) {
    HIP_OK(hipEventRecord(s.ev_side, s.side));
    HIP_OK(hipStreamWaitEvent(s.stream, s.ev_side, 0));
  }
  if (s.side_pending & 2) {
    HIP_OK(hipEventRecord(s.ev_side2, s.side2));
    HIP_OK(hipStreamWaitEvent(s.stream, s.ev_side2, 0));
  }
  s.side_pending = 0;
}

// ---------------------------- device error flags ----------------------------
// Every failure a kernel can detect is a device word the host reads once the work is done
// (nothing throws inside a launch): a Cholesky factor that is not positive definite
// (dev_flags[0] the per-species / per-unit / GammaEta / spatial systems, [1] updateGamma2,
// [2] the phylogeny BetaLambda system), and every bounded in-launch handshake that timed out
// (the Gamma2 / BetaLambda launch's gbl_sync[3]; the dense solver's error word, whose bits
// name the wait, state.h HsErr).  A timed-out wait lets its launch drain on stale data, so a
// run that saw one must fail, never return its samples.  Called with the streams idle.
// zero the error words (not the handshake state): an error is reported by the one call that
// saw it, and the chain can be read, reset with set_state / init_state and run again
static void clear_device_errors(State& s) {
  HIP_OK(hipMemsetAsync(s.dev_flags, 0, 3 * sizeof(int), s.stream));
  HIP_OK(hipMemsetAsync(s.gbl_sync + 3, 0, sizeof(int), s.stream));
  HIP_OK(hipMemsetAsync(s.trsv_sync + DENSE_SYNC_ERR, 0, sizeof(int), s.stream));
  HIP_OK(hipStreamSynchronize(s.stream));
}

static void check_device_flags(State& s) {
  // one copy of the error block (build_state): dev_flags, gbl_sync, the dense handshake words
  int blk[20 + DENSE_SYNC_ERR + 1] = {0};
  copy_sync(blk, s.dev_flags, sizeof(blk), hipMemcpyDeviceToHost, s.stream);
  const int* flag = blk;
  const int* gsync = blk + 16;
  const int hs = blk[20 + DENSE_SYNC_ERR];
  if (flag[0] || flag[1] || flag[2] || gsync[3] || hs) clear_device_errors(s);  // reported once
  if (hs != 0) {
    std::string what;
    if (hs & HS_ERR_TRSV_FLAG) what += " [sync-free triangular solve: a block flag never came up]";
    if (hs & HS_ERR_TRSV_TICKET) what += " [sync-free triangular solve: corrupt block ticket]";
    if (hs & HS_ERR_CHOL_PANEL) what += " [blocked Cholesky: the fused panel step's diagonal-inverse flag never came up]";
    throw HmscError(-5, "internal: an in-launch handshake of the blocked dense solver timed out; the sweep used a "
                        "half-solved system and its draws are invalid" + what);
  }
  if (gsync[3] != 0)
    throw HmscError(-5, "internal: the Gamma2 / BetaLambda in-launch handshake timed out; the sweep's draws are invalid");
  if (flag[2] != 0)
    throw HmscError(-1, "a Cholesky factorisation failed in the phylogeny BetaLambda system (matrix not positive definite)");
  if (flag[1] != 0) throw HmscError(-1, "a Cholesky factorisation failed in updateGamma2 (matrix not positive definite)");
  if (flag[0] != 0) throw HmscError(-1, "a Cholesky factorisation failed (matrix not positive definite)");
}

// ---------------------------- state get / set ----------------------------
static void get_state(State& s, hmsc_params* p) {
  DeviceGuard dg(s.device);
  join_side(s);
  HIP_OK(hipStreamSynchronize(s.stream));
  check_device_flags(s);
  const int K = s.K, nsl = s.nsl, nc = s.nc;
  std::vector<double> BL((size_t)K * nsl), Psi((size_t)s.NF * nsl), Delta(std::max(1, s.NF));
  d2h(BL.data(), s.BL, BL.size(), s.stream);
  d2h(Psi.data(), s.Psi, Psi.size(), s.stream);
  d2h(Delta.data(), s.Delta, s.NF, s.stream);
  if (p->Gamma) d2h(p->Gamma, s.Gamma, (size_t)nc * s.nt, s.stream);
  if (p->iV) d2h(p->iV, s.iV, (size_t)nc * nc, s.stream);
  if (p->iSigma) d2h(p->iSigma, s.iSigma, nsl, s.stream);
  if (p->Z) d2h(p->Z, s.Z, (size_t)s.ny * nsl, s.stream);
  for (int r = 0; r < s.nr; ++r) {
    p->nf[r] = s.lev[r].nf;
    if (p->Eta[r]) d2h(p->Eta[r], s.lev[r].Eta, (size_t)s.lev[r].np * s.lev[r].nf, s.stream);
  }
  HIP_OK(hipStreamSynchronize(s.stream));
  if (p->Beta)
    for (int j = 0; j < nsl; ++j)
      for (int c = 0; c < nc; ++c) p->Beta[c + (size_t)nc * j] = BL[c + (size_t)K * j];
  for (int r = 0; r < s.nr; ++r) {
    const int nf = s.lev[r].nf, lo = s.loff(r), fo = s.foff(r);
    for (int j = 0; j < nsl; ++j)
      for (int h = 0; h < nf; ++h) {
        if (p->Lambda[r]) p->Lambda[r][h + (size_t)nf * j] = BL[lo + h + (size_t)K * j];
        if (p->Psi[r]) p->Psi[r][h + (size_t)nf * j] = Psi[fo + h + (size_t)s.NF * j];
      }
    std::vector<double> ad(std::max(1, nf), 1.0);
    if (nf > 0) copy_sync(ad.data(), s.lev[r].AlphaD, sizeof(double) * nf, hipMemcpyDeviceToHost, s.stream);
    for (int h = 0; h < nf; ++h) {
      if (p->Delta[r]) p->Delta[r][h] = Delta[fo + h];
      if (p->Alpha[r]) p->Alpha[r][h] = (int32_t)ad[h];
    }
  }
  double rho = 1.0;
  copy_sync(&rho, s.rho, sizeof(double), hipMemcpyDeviceToHost, s.stream);
  p->rho = (int32_t)rho;
}

static void set_state(State& s, const hmsc_params* p) {
  DeviceGuard dg(s.device);
  join_side(s);
  HIP_OK(hipStreamSynchronize(s.stream));
  clear_device_errors(s);  // a new state: earlier failures are not its own
  // the device holds BL / Psi / Delta in the current layout (K, NF and the per-level row
  // offsets); read them in that layout, then remap every level's rows to the new nf (rows a
  // level gains: Lambda 0, Psi 1, Delta 1) before the supplied fields are applied
  const int K0 = s.K, NF0 = s.NF, nsl = s.nsl, nc = s.nc;
  std::vector<int> lo0(s.nr), fo0(s.nr), nf0(s.nr);
  for (int r = 0; r < s.nr; ++r) lo0[r] = s.loff(r), fo0[r] = s.foff(r), nf0[r] = s.lev[r].nf;
  std::vector<double> BL0((size_t)K0 * nsl), Psi0((size_t)std::max(1, NF0) * nsl), Delta0(std::max(1, NF0));
  d2h(BL0.data(), s.BL, BL0.size(), s.stream);
  d2h(Psi0.data(), s.Psi, (size_t)NF0 * nsl, s.stream);
  d2h(Delta0.data(), s.Delta, NF0, s.stream);
  HIP_OK(hipStreamSynchronize(s.stream));
  for (int r = 0; r < s.nr; ++r) {
    if (p->nf[r] > 0) {
      HMSC_REQUIRE(p->nf[r] <= s.lev[r].nfcap, "set_state: nf exceeds the level's factor capacity (hmsc_get_nf_cap)");
      s.lev[r].nf = p->nf[r];
    }
  }
  s.refresh_dims();
  HMSC_REQUIRE(s.K <= s.Kmax, "set_state: K = nc + sum(nf) exceeds the chain's capacity (<= 128)");
  const int K = s.K;
  std::vector<double> BL((size_t)K * nsl, 0.0), Psi((size_t)std::max(1, s.NF) * nsl, 1.0), Delta(std::max(1, s.NF), 1.0);
  for (int j = 0; j < nsl; ++j)
    for (int c = 0; c < nc; ++c) BL[c + (size_t)K * j] = BL0[c + (size_t)K0 * j];
  for (int r = 0; r < s.nr; ++r) {
    const int keep = std::min(nf0[r], s.lev[r].nf), lo = s.loff(r), fo = s.foff(r);
    for (int h = 0; h < keep; ++h) {
      for (int j = 0; j < nsl; ++j) {
        BL[lo + h + (size_t)K * j] = BL0[lo0[r] + h + (size_t)K0 * j];
        Psi[fo + h + (size_t)s.NF * j] = Psi0[fo0[r] + h + (size_t)NF0 * j];
      }
      Delta[fo + h] = Delta0[fo0[r] + h];
    }
  }
  if (p->Beta)
    for (int j = 0; j < nsl; ++j)
      for (int c = 0; c < nc; ++c) BL[c + (size_t)K * j] = p->Beta[c + (size_t)nc * j];
  for (int r = 0; r < s.nr; ++r) {
    const int nf = s.lev[r].nf, lo = s.loff(r), fo = s.foff(r);
    for (int j = 0; j < nsl; ++j)
      for (int h = 0; h < nf; ++h) {
        if (p->Lambda[r]) BL[lo + h + (size_t)K * j] = p->Lambda[r][h + (size_t)nf * j];
        if (p->Psi[r]) Psi[fo + h + (size_t)s.NF * j] = p->Psi[r][h + (size_t)nf * j];
      }
    if (p->Delta[r])
      for (int h = 0; h < nf; ++h) Delta[fo + h] = p->Delta[r][h];
    if (p->Eta[r]) h2d(s.lev[r].Eta, p->Eta[r], (size_t)s.lev[r].np * nf, s.stream);
    if (p->Alpha[r] && nf > 0) {  // initPar$Alpha (R/computeInitialParameters.R:212-221)
      std::vector<double> ad(nf);
      for (int h = 0; h < nf; ++h) {
        HMSC_REQUIRE(p->Alpha[r][h] >= 1 && (!s.lev[r].spatial || p->Alpha[r][h] <= s.lev[r].nalpha),
                     "set_state: Alpha index out of the alphapw grid");
        ad[h] = s.lev[r].spatial ? p->Alpha[r][h] : 1.0;
      }
      copy_sync(s.lev[r].AlphaD, ad.data(), sizeof(double) * nf, hipMemcpyHostToDevice, s.stream);
    }
  }
  h2d(s.BL, BL.data(), BL.size(), s.stream);
  h2d(s.Psi, Psi.data(), (size_t)s.NF * nsl, s.stream);
  h2d(s.Delta, Delta.data(), s.NF, s.stream);
  if (p->Gamma) h2d(s.Gamma, p->Gamma, (size_t)nc * s.nt, s.stream);
  if (p->iV) h2d(s.iV, p->iV, (size_t)nc * nc, s.stream);
  if (p->iSigma) {
    h2d(s.iSigma, p->iSigma, nsl, s.stream);
    s.isigma_fixed_one = false;  // an initPar sigma: updateGamma2 checks iSigma == 1 again
  }
  if (p->Z) h2d(s.Z, p->Z, (size_t)s.ny * nsl, s.stream);
  if (p->rho > 0) {  // initPar$rho as a grid index (R/computeInitialParameters.R:223-224)
    HMSC_REQUIRE(!s.phylo || p->rho <= s.nrho, "set_state: rho index out of range");
    const double rho = p->rho;
    copy_sync(s.rho, &rho, sizeof(double), hipMemcpyHostToDevice, s.stream);
  }
  HIP_OK(hipStreamSynchronize(s.stream));
  s.zt_valid = false;
  s.xz_parts = 0;
  s.xeta_valid = false;
  s.g2prep_valid = false;
  s.g2s_valid = false;
  s.graph_dirty = true;
}

// ---------------------------- updateNf (host decision) ----------------------------
// R/updateNf.R:3-70: with probability exp(-(1 + 0.0005 iter)) add a factor (if none is
// redundant) or drop (reference quirk: setdiff(1:nf, logical) drops factor 1).  A
// covariate-dependent level's group (Level::xgroup levels from r sharing Eta, Lambda[,,k] in
// level r + k) adapts together: the redundancy counts run over every k (rowMeans of the nf x ns
// x ncr array), a new factor adds a row to every Lambda[,,k] / Psi[,,k] / Delta[,k] (:41-47)
// and one Eta column, a dropped factor leaves all of them (:62-66).
static void update_nf(State& s, int r, uint32_t iter) {
  Level& L = s.lev[r];
  if (L.eta_alias()) return;  // (adapted with its group's first level)
  const int m = L.xgroup;
  const uint32_t st = LEVEL_STRIDE * r;
  const double u = uniforms(s.key, 0, 0, S_NF + st, iter).a;
  const double prob = 1.0 / std::exp(1.0 + 0.0005 * iter);
  if (!(u < prob)) return;
  HIP_OK(hipStreamSynchronize(s.stream));
  const int K = s.K, NF = s.NF, nsl = s.nsl, nf = L.nf;
  std::vector<int> lo0(s.nr), fo0(s.nr);
  for (int q = 0; q < s.nr; ++q) lo0[q] = s.loff(q), fo0[q] = s.foff(q);
  std::vector<double> BL((size_t)K * nsl);
  d2h(BL.data(), s.BL, BL.size(), s.stream);
  HIP_OK(hipStreamSynchronize(s.stream));
  std::vector<double> small(nf, 0.0);
  for (int k = 0; k < m; ++k)
    for (int j = 0; j < nsl; ++j)
      for (int h = 0; h < nf; ++h) small[h] += std::fabs(BL[lo0[r + k] + h + (size_t)K * j]) < 1e-3 ? 1.0 : 0.0;
  if (s.sharded) {  // the counts over every rank's species (an adaptation sweep's extra all-reduce)
    h2d(s.allreduce_buf, small.data(), nf, s.stream);
    ar_point(s, s.allreduce_buf, nf);
    d2h(small.data(), s.allreduce_buf, nf, s.stream);
    HIP_OK(hipStreamSynchronize(s.stream));
  }
  int num_red = 0;
  bool all_lt = true;
  for (int h = 0; h < nf; ++h) {
    const double prop = small[h] / ((double)s.ns * m);
    if (prop >= 1.0) ++num_red;
    if (!(prop < 0.995)) all_lt = false;
  }
  int grow = 0;  // +1 add a factor, -1 drop factor 1
  if (nf < L.nfmax && iter > 20 && num_red == 0 && all_lt) {
    if (nf + 1 > L.nfcap || s.K + m > s.Kmax)
      throw HmscError(-6, "updateNf: level " + std::to_string(r + 1) + " needs " + std::to_string(nf + 1) +
                              " latent factors at iteration " + std::to_string(iter) + ", but this build holds at most " +
                              std::to_string(L.nfcap) + " for it (K = nc + sum(nf) <= 128); set nfMax <= " +
                              std::to_string(L.nfcap) + " with setPriors (or fewer covariates) to run this model");
    grow = 1;
  } else if (num_red > 0 && nf > L.nfmin) {
    grow = -1;
  } else {
    return;
  }
  std::vector<double> Psi((size_t)NF * nsl), Delta(std::max(1, NF)), Eta((size_t)L.np * nf);
  d2h(Psi.data(), s.Psi, Psi.size(), s.stream);
  d2h(Delta.data(), s.Delta, NF, s.stream);
  d2h(Eta.data(), L.Eta, Eta.size(), s.stream);
  HIP_OK(hipStreamSynchronize(s.stream));
  for (int k = 0; k < m; ++k) s.lev[r + k].nf = nf + grow;
  s.refresh_dims();
  const int K2 = s.K, NF2 = s.NF;
  std::vector<double> BL2((size_t)K2 * nsl), Psi2((size_t)std::max(1, NF2) * nsl), Delta2(std::max(1, NF2));
  for (int j = 0; j < nsl; ++j)
    for (int c = 0; c < s.nc; ++c) BL2[c + (size_t)K2 * j] = BL[c + (size_t)K * j];
  for (int q = 0; q < s.nr; ++q) {
    const bool in = q >= r && q < r + m;
    const Level& Lq = s.lev[q];
    const int lo2 = s.loff(q), fo2 = s.foff(q);
    for (int h = 0; h < Lq.nf; ++h) {
      // the old row of new row h: the same (other levels; kept factors), the next one (the
      // dropped factor 1, :56), or none (the added factor)
      const int ho = !in ? h : grow > 0 ? (h < nf ? h : -1) : h + 1;
      for (int j = 0; j < nsl; ++j) {
        BL2[lo2 + h + (size_t)K2 * j] = ho >= 0 ? BL[lo0[q] + ho + (size_t)K * j] : 0.0;  // rbind(lambda, 0) (:33)
        Psi2[fo2 + h + (size_t)NF2 * j] =
            ho >= 0 ? Psi[fo0[q] + ho + (size_t)NF * j]
                    : gamma_std(s.key, (uint32_t)(s.sp0 + j), S_NF_PSI + LEVEL_STRIDE * q, iter, Lq.nu / 2) / (Lq.nu / 2);  // (:36,44)
      }
      Delta2[fo2 + h] = ho >= 0 ? Delta[fo0[q] + ho]
                                : gamma_std(s.key, 0, S_NF_DELTA + LEVEL_STRIDE * q, iter, Lq.a2) / Lq.b2;  // (:39,47)
    }
  }
  h2d(s.BL, BL2.data(), BL2.size(), s.stream);
  h2d(s.Psi, Psi2.data(), (size_t)NF2 * nsl, s.stream);
  h2d(s.Delta, Delta2.data(), NF2, s.stream);
  if (grow > 0) {
    std::vector<double> col(L.np);
    for (int q = 0; q < L.np; ++q) col[q] = normal(s.key, (uint32_t)q, 0, S_NF_ETA + st, iter);  // (:30)
    h2d(L.Eta + (size_t)L.np * nf, col.data(), L.np, s.stream);
    const double one = 1.0;  // alphaNew = c(alpha, 1)  (:31)
    for (int k = 0; k < m; ++k) h2d(s.lev[r + k].AlphaD + nf, &one, 1, s.stream);
  } else {
    h2d(L.Eta, Eta.data() + L.np, (size_t)L.np * (nf - 1), s.stream);  // eta[, indNotRed] (:57)
    for (int k = 0; k < m; ++k) {  // alpha = alpha[indNotRed]  (:59)
      std::vector<double> ad(nf);
      d2h(ad.data(), s.lev[r + k].AlphaD, nf, s.stream);
      HIP_OK(hipStreamSynchronize(s.stream));
      if (nf > 1) h2d(s.lev[r + k].AlphaD, ad.data() + 1, nf - 1, s.stream);
    }
  }
  HIP_OK(hipStreamSynchronize(s.stream));
  s.zt_valid = false;
  s.xz_parts = 0;
  s.xeta_valid = false;
  s.g2s_valid = false;
  s.graph_dirty = true;
}

// ---------------------------- sweep ----------------------------
static void run_updater(State& s, uint32_t which, uint32_t iter) {
  if (s.sharded) {
    run_updater_sharded(s, which, iter);
    return;
  }
  switch (which) {
    case HMSC_UP_GAMMA2:
      launch_gamma2(s, iter);
      break;
    case HMSC_UP_GAMMAETA:
      join_side(s);  // reads iV (GammaV) and Eta of the previous sweep
      launch_gamma_eta(s, iter);
      break;
    case HMSC_UP_BETALAMBDA:
      launch_beta_lambda(s, iter);
      break;
    case HMSC_UP_GAMMAV:
      launch_gamma_v(s, iter, s.stream);
      break;
    case HMSC_UP_RHO:
      if (s.phylo) launch_rho(s, iter, s.stream);  // only with C (R/sampleMcmc.R:263)
      break;
    case HMSC_UP_LAMBDAPRIORS:
      launch_lambda_priors(s, iter, s.stream);
      break;
    case HMSC_UP_ETA:
      launch_eta(s, iter);
      break;
    case HMSC_UP_ALPHA:
      launch_alpha(s, iter);  // spatial 'Full' levels; rep(1, nf) otherwise (R/updateAlpha.R:81-82)
      break;
    case HMSC_UP_INVSIGMA:
      launch_inv_sigma(s, iter);
      break;
    case HMSC_UP_Z:
      launch_update_z(s, iter, false);
      break;
    default:
      throw HmscError(-1, "unknown or out-of-scope updater bit");
  }
}

// One sweep in the reference order (R/sampleMcmc.R:219-306).  updateGammaV and
// updateLambdaPriors of sweep t only feed sweep t+1 (Gamma2 / BetaLambda and the record),
// so they run on the side stream after BetaLambda, overlapped with Eta / InvSigma / Z.
static void sweep(State& s, uint32_t iter, bool adapt) {
  if (s.sharded) {
    sweep_sharded(s, iter);  // kernels.hip: two all-reduces per sweep
    if (adapt) {
      join_side(s);
      for (int r = 0; r < s.nr; ++r) update_nf(s, r, iter);
    }
    return;
  }
  ProfScope ps(s, PROF_SWEEP);
  // co-launched side updaters (launch_side_fused): the GammaV algebra of the previous sweep
  // may still run on the side stream; Gamma2 joins it before its final stage
  const bool fused = s.nranks == 1 && side_fusion_ok(s);
  if (!fused) join_side(s);
  if (gamma2_bl_fusion_ok(s)) {
    launch_gamma2_bl(s, iter);  // both updaters in one launch (BetaLambda's factorization overlaps Gamma2)
  } else {
    if (s.mask & HMSC_UP_GAMMA2) run_updater(s, HMSC_UP_GAMMA2, iter);
    if (s.mask & HMSC_UP_GAMMAETA) run_updater(s, HMSC_UP_GAMMAETA, iter);
    join_side(s);  // BetaLambda reads Gamma and iV
    if (s.mask & HMSC_UP_BETALAMBDA) run_updater(s, HMSC_UP_BETALAMBDA, iter);
  }
  s.side_fused = fused;
  if (fused) {
    launch_side_fused(s, iter);
    for (uint32_t u : {HMSC_UP_ALPHA, HMSC_UP_INVSIGMA, HMSC_UP_Z})
      if (s.mask & u) run_updater(s, u, iter);
  } else {
    // (sharded chains keep every RCCL collective on one stream: no side-stream overlap)
    const bool side_work = s.nranks == 1 && !s.single_stream && !s.phylo && (s.mask & (HMSC_UP_GAMMAV | HMSC_UP_LAMBDAPRIORS)) != 0;
    if (side_work) {
      HIP_OK(hipEventRecord(s.ev_bl, s.stream));
      HIP_OK(hipStreamWaitEvent(s.side, s.ev_bl, 0));
      HIP_OK(hipStreamWaitEvent(s.side2, s.ev_bl, 0));
      if (s.mask & HMSC_UP_GAMMAV) launch_gamma_v(s, iter, s.side);
      if (s.mask & HMSC_UP_LAMBDAPRIORS) launch_lambda_priors(s, iter, s.side2);
      s.side_pending = 3;
    } else {
      if (s.mask & HMSC_UP_GAMMAV) launch_gamma_v(s, iter, s.stream);
      if ((s.mask & HMSC_UP_RHO) && s.phylo) launch_rho(s, iter, s.stream);  // R/sampleMcmc.R:263-266
      if (s.mask & HMSC_UP_LAMBDAPRIORS) launch_lambda_priors(s, iter, s.stream);
    }
    for (uint32_t u : {HMSC_UP_ETA, HMSC_UP_ALPHA, HMSC_UP_INVSIGMA, HMSC_UP_Z})
      if (s.mask & u) run_updater(s, u, iter);
  }
  if (adapt) {
    join_side(s);
    for (int r = 0; r < s.nr; ++r) update_nf(s, r, iter);
  }
}

// ---------------------------- sweep hipGraphs ----------------------------
// Steady-state sweeps (no updateNf, one rank) are captured once into graphs of
// s.graph_sweeps consecutive sweeps and replayed: one launch per graph_sweeps sweeps instead
// of ~20 kernel launches + event records per sweep, and the relaunch gap between replays is
// paid once per replay.  Kernels captured with s.capturing read the Philox sweep counter
// from s.d_iter, which for the i-th captured sweep is slot i of s.d_iters; one small kernel
// writes iter .. iter + n - 1 into the slots before each replay.  gx[1][k] is the same
// sequence with the record pack after every sweep; the pack picks its ring slot (or returns,
// for a sweep that is not recorded) from d_iter and the run descriptor d_rec_desc.
// Pack the state after a sweep into a ring slot (nullptr: chosen on the device in a graph
// replay).  With co-launched side updaters the side stream's outputs are packed on it, so
// the main stream need not wait for the GammaV algebra.
static void record_after_sweep(State& s, double* slot) {
  if (s.ext_pending && s.capturing && s.cap_sweep == 0) {  // the first sweep's side work is external
    if (!s.pack_done) launch_record(s, slot, 1);
    ext_add_record(s);
  } else if ((s.side_fused || sharded_pack_split(s)) && (s.side_pending & 1)) {
    if (!s.pack_done) launch_record(s, slot, 1);  // else updateZ's slab-sum launch packed it
    launch_record(s, slot, 2);
  } else {
    join_side(s);
    launch_record(s, slot, 0);
  }
  s.pack_req = s.pack_done = false;
}

__global__ void set_iters_kernel(uint32_t* p, uint32_t v, int n, unsigned long long* kt = nullptr) {
  if ((int)threadIdx.x < n) p[threadIdx.x] = v + threadIdx.x;
  if (kt && threadIdx.x == 0) kt_record(kt, v, kt_now());  // the replay's start (KT_IT)
}
static unsigned long long* kt_iters(const State& s) {
  return s.kt_on ? s.d_kt + (size_t)KT_IT * 2 * KT_SLOTS : nullptr;
}
// A run's start in one launch instead of a descriptor kernel and three fills (~25 us of the
// 20-sweep line): the record descriptor, and the device flags a run resets -- the fused
// Gamma2 + BetaLambda launch's epoch words, the tails' CR / W flag and the side chain's flags
// (a run's sweeps are distinct, but an earlier run may have ended on one of them)
__global__ void run_start_kernel(int32_t* desc, int32_t iter0, int32_t transient, int32_t thin, int32_t samples,
                                 int* gbl, int* crw, int* side, int nside, int32_t nonce) {
  const int t = threadIdx.x;
  if (desc && t < 5) desc[t] = t == 0 ? iter0 : t == 1 ? transient : t == 2 ? thin : t == 3 ? samples : nonce;
  if (gbl && (t == 4 || t == 5)) gbl[t - 3] = 0;
  if (crw && t == 6) crw[0] = 0;
  if (side && t >= 8 && t < 8 + nside) side[t - 8] = 0;
}

static void destroy_graph(State& s) {
  for (auto& row : s.gx)
    for (hipGraphExec_t& g : row) {
      if (g) (void)hipGraphExecDestroy(g);
      g = nullptr;
    }
  for (auto& row : s.ext_side)
    for (auto& f : row) f = nullptr;
  for (auto& v : s.gseg) {
    for (auto& g : v)
      if (g.g) (void)hipGraphExecDestroy(g.g);
    v.clear();
  }
}

// a sharded chain on a host transport: its sweep graphs are segments split at the all-reduces
static bool host_segments(const State& s) { return s.sharded && s.comm == nullptr; }

// Captures graph_sweeps sweeps (with or without the record pack after each).  Returns
// nullptr when the sweep is not in a steady state, i.e. the host-side validity flags it
// changes would differ on the next sweep.  segs (a host-transport sharded chain): the sweep is
// captured as segments split at its all-reduces (ar_point), instantiated into *segs; the
// return value is then null.
static hipGraphExec_t capture_sweeps(State& s, uint32_t iter, bool with_record, size_t* n_nodes = nullptr,
                                     int nsweeps = 0, std::vector<State::Seg>* segs = nullptr) {
  if (nsweeps <= 0) nsweeps = s.graph_sweeps;
  std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
  join_side(s);
  const bool xv = s.xeta_valid, zv = s.zt_valid, gv = s.g2prep_valid, gp = s.g_pending, g2v = s.g2s_valid;
  const int xzp = s.xz_parts;
  hipGraph_t g = nullptr;
  std::vector<std::pair<hipGraph_t, size_t>> parts;  // (host transport) the segments so far
  auto drop_parts = [&] {
    for (auto& pr : parts)
      if (pr.first) (void)hipGraphDestroy(pr.first);
    parts.clear();
  };
  HIP_OK(hipStreamBeginCapture(s.stream, hipStreamCaptureModeThreadLocal));
  s.capturing = true;
  s.side_root = false;
  s.ar_in_capture = 0;
  s.cap_segs = segs ? &parts : nullptr;
  try {
    const char* no_root = std::getenv("HMSC_NO_SIDE_ROOT");
    s.edge_free_now = s.edge_free && live_chains(s.device) == 1;
    // (a sharded RCCL chain: sweep_sharded's edge-free sweeps fork and join on the device too)
    const bool shard_root = s.sharded && s.comm != nullptr && !s.single_stream && sharded_fused_ok(s) &&
                            !getenv_flag("HMSC_NO_SHARD_DEV");
    if (((s.side_fused && !s.sharded) || shard_root) && s.edge_free_now && !(no_root && no_root[0] == '1')) {
      // the side stream forked at the graph's root: the first sweep's side work then waits for
      // the fused launch's tails flag on the device like the later sweeps', instead of behind a
      // graph edge from that launch (whose first replay sweep's side chain ended ~100 us late)
      HIP_OK(hipEventRecord(s.ev_bl, s.stream));
      HIP_OK(hipStreamWaitEvent(s.side, s.ev_bl, 0));
      s.side_pending |= 1;
      s.side_root = true;
    }
    int pmask = 0;
    s.cap_kcopy = s.kcopy && with_record && nsweeps <= s.kcopy_max;
    for (int i = 0; i < nsweeps; ++i) {
      s.d_iter = s.d_iters + i;
      s.cap_sweep = i;
      s.pack_req = with_record;
      s.pack_done = false;
      s.cap_pack_mask = 0;
      sweep(s, iter, false);
      if (with_record) record_after_sweep(s, nullptr);
      pmask = i == 0 ? s.cap_pack_mask : (pmask == s.cap_pack_mask ? pmask : -1);
    }
    s.gx_pack_mask[with_record ? 1 : 0][graph_level(nsweeps)] = s.cap_kcopy ? pmask : 0;
    s.cap_kcopy = false;
    s.d_iter = s.d_iters;
    s.cap_sweep = -1;
    s.side_root = false;
    join_side(s);
  } catch (...) {
    s.cap_sweep = -1;
    s.side_root = false;
    s.cap_kcopy = false;
    s.ext_pending = nullptr;
    s.d_iter = s.d_iters;
    s.pack_req = s.pack_done = false;
    s.capturing = false;
    s.cap_segs = nullptr;
    s.edge_free_now = false;
    (void)hipStreamEndCapture(s.stream, &g);
    if (g) (void)hipGraphDestroy(g);
    drop_parts();
    s.xeta_valid = xv, s.zt_valid = zv, s.g2prep_valid = gv, s.g_pending = gp, s.g2s_valid = g2v;
    s.xz_parts = xzp;
    throw;
  }
  s.capturing = false;
  s.cap_segs = nullptr;
  // (also a graph captured while the chain was alone on its device: its fused launch may have
  // taken the resident-slot layout that two overlapping launches cannot share, kernels.hip)
  s.graph_edge_free = s.edge_free_now || live_chains(s.device) == 1;
  s.edge_free_now = false;
  HIP_OK(hipStreamEndCapture(s.stream, &g));
  const bool steady = xv == s.xeta_valid && zv == s.zt_valid && gv == s.g2prep_valid && gp == s.g_pending &&
                      g2v == s.g2s_valid && xzp == s.xz_parts;
  s.xeta_valid = xv, s.zt_valid = zv, s.g2prep_valid = gv, s.g_pending = gp, s.g2s_valid = g2v;  // nothing ran yet
  s.xz_parts = xzp;
  if (s.sharded && !with_record) s.ar_per_graph_sweep = s.ar_in_capture / std::max(1, nsweeps);
  size_t nodes = 0;
  HIP_OK(hipGraphGetNodes(g, nullptr, &nodes));
  for (auto& pr : parts) {
    size_t k = 0;
    HIP_OK(hipGraphGetNodes(pr.first, nullptr, &k));
    nodes += k;
  }
  if (n_nodes) *n_nodes = nodes;
  if (const char* e = std::getenv("HMSC_GRAPH_DEBUG"))
    if (e[0] == '1')
      std::fprintf(stderr, "[hmsc] captured %d sweeps%s: %zu nodes in %zu segment(s)%s\n", nsweeps,
                   with_record ? " + record" : "", nodes, parts.size() + 1, steady ? "" : " (not steady)");
  hipGraphExec_t ge = nullptr;
  if (segs) {
    parts.emplace_back(g, 0);  // the last segment: no all-reduce after it
    g = nullptr;
    segs->clear();
    if (steady && nodes <= graph_max_nodes()) {
      try {
        for (size_t k = 0; k < parts.size(); ++k) {
          State::Seg sg;
          HIP_OK(hipGraphInstantiate(&sg.g, parts[k].first, nullptr, nullptr, 0));
          sg.ar_n = parts[k].second;
          segs->push_back(sg);
        }
      } catch (...) {
        for (auto& sg : *segs)
          if (sg.g) (void)hipGraphExecDestroy(sg.g);
        segs->clear();
        drop_parts();
        throw;
      }
    }
    drop_parts();
    return nullptr;
  }
  if (steady && nodes <= graph_max_nodes()) HIP_OK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  HIP_OK(hipGraphDestroy(g));
  // the first sweep's side work, if it was left out of the graph, goes with it
  s.ext_side[with_record ? 1 : 0][graph_level(nsweeps)] = ge ? std::move(s.ext_pending) : nullptr;
  s.ext_pending = nullptr;
  return ge;
}

// Graphs of graph_sweeps, graph_sweeps / 2, ..., 1 sweeps, with and without the record pack:
// a run of n sweeps replays n's binary decomposition (at most log2(graph_sweeps) + 1 replays
// for the remainder, instead of one replay per remaining sweep).
static bool build_sweep_graphs(State& s, uint32_t iter) {
  destroy_graph(s);
  size_t nodes = 0;
  if (host_segments(s)) {  // one sweep per replay, as segments (the host sums between them)
    s.graph_sweeps = 1;
    capture_sweeps(s, iter, false, &nodes, 1, &s.gseg[0]);
    if (!s.gseg[0].empty()) capture_sweeps(s, iter, true, nullptr, 1, &s.gseg[1]);
    if (s.gseg[0].empty() || s.gseg[1].empty()) {
      if (nodes > graph_max_nodes()) s.use_graph = false;
      destroy_graph(s);
      return false;
    }
    s.graph_K = s.K;
    s.graph_NF = s.NF;
    s.graph_dirty = false;
    return true;
  }
  const int top = graph_level(s.graph_sweeps);
  s.gx[0][top] = capture_sweeps(s, iter, false, &nodes);
  if (!s.gx[0][top] && nodes > graph_max_nodes() && s.graph_sweeps > 1) {
    // a sweep with many launches (dense phylogeny / spatial factorizations): fewer sweeps
    // per graph, or none when one sweep alone exceeds the cap (its launch overhead is hidden
    // behind milliseconds of device work anyway)
    const size_t per_sweep = (nodes + s.graph_sweeps - 1) / s.graph_sweeps;
    const int fit = (int)std::max<size_t>(1, graph_max_nodes() / (per_sweep + 4));  // + the record pack
    s.graph_sweeps = 1 << graph_level(fit);
    s.gx[0][graph_level(s.graph_sweeps)] = capture_sweeps(s, iter, false, &nodes);
  }
  const int lv = graph_level(s.graph_sweeps);
  if (!s.gx[0][lv]) {
    if (nodes > graph_max_nodes()) s.use_graph = false;  // eager from here on
    return false;
  }
  for (int k = lv; k >= 0; --k) {
    if (k < lv) s.gx[0][k] = capture_sweeps(s, iter, false, nullptr, 1 << k);
    if (s.gx[0][k]) s.gx[1][k] = capture_sweeps(s, iter, true, nullptr, 1 << k);
    if (!s.gx[0][k] || !s.gx[1][k]) {
      if (k == lv) {
        destroy_graph(s);
        return false;
      }
      break;  // smaller remainders run eagerly
    }
  }
  s.graph_K = s.K;
  s.graph_NF = s.NF;
  s.graph_dirty = false;
  return true;
}

static bool graphs_built(const State& s) {
  return host_segments(s) ? !s.gseg[0].empty() : s.gx[0][graph_level(s.graph_sweeps)] != nullptr;
}

// Runs sweeps iter .. iter+n-1 (n a power of two <= graph_sweeps) as one
// graph replay if the graphs exist or can be built now; returns false (nothing launched) when
// the caller must run eagerly.
static bool replay_sweeps(State& s, uint32_t iter, bool with_record, int n) {
  if (!s.use_graph || s.prof) return false;
  if (graphs_built(s) && s.graph_edge_free && live_chains(s.device) > 1) s.graph_dirty = true;  // recapture with edges
  if (graphs_built(s) && (s.graph_dirty || s.graph_K != s.K || s.graph_NF != s.NF)) destroy_graph(s);
  if (s.graph_dirty) s.eager_streak = 0, s.graph_dirty = false;
  if (!graphs_built(s) && (s.eager_streak < 1 || !build_sweep_graphs(s, iter))) return false;  // steady first
  if (n < 1 || n > s.graph_sweeps || (n & (n - 1))) return false;
  if (host_segments(s)) {
    const auto& segs = s.gseg[with_record ? 1 : 0];
    if (segs.empty() || n != 1) return false;
    join_side(s);
    set_iters_kernel<<<1, 64, 0, s.stream>>>(s.d_iters, iter, n, kt_iters(s));
    for (const auto& sg : segs) {
      HIP_OK(hipGraphLaunch(sg.g, s.stream));
      if (sg.ar_n) {  // the segment ended with the D2H copy of the all-reduce buffer; the next one starts with its H2D
        HIP_OK(hipStreamSynchronize(s.stream));
        ++s.ar_calls;
        s.ar_doubles += sg.ar_n;
        HMSC_REQUIRE(s.host_allreduce(s.ar_host, (int64_t)sg.ar_n, s.host_allreduce_ctx) == 0,
                     "host all-reduce callback failed");
      }
    }
    return true;
  }
  hipGraphExec_t ge = s.gx[with_record ? 1 : 0][graph_level(n)];
  if (!ge) return false;
  // the live-chain recheck and the launch under one lock: a chain created since the check above
  // would run next to an edge-free graph's device-side joins (build_state drains the device
  // when a device's count reaches 2, so the replays queued before that have finished)
  std::unique_lock<std::recursive_mutex> dev_lock(g_dev_mu);
  if (s.graph_edge_free && live_chains(s.device) > 1) {
    dev_lock.unlock();
    destroy_graph(s);  // this sweep runs eagerly; the graphs are recaptured with edges after it
    s.graph_dirty = false;
    s.eager_streak = 0;
    return false;
  }
  join_side(s);
  set_iters_kernel<<<1, 64, 0, s.stream>>>(s.d_iters, iter, n, kt_iters(s));
  if (const auto& ext = s.ext_side[with_record ? 1 : 0][graph_level(n)]) {
    // the replay's first side chain, on the side stream ahead of the graph (State::ext_side):
    // it waits on the device for that sweep's tails flag like the graph's own side chains
    // (behind the replay's start on the main stream: enqueued early, it would otherwise hold
    // its CU slots spinning through the previous replay)
    HIP_OK(hipEventRecord(s.ev_ext_go, s.stream));
    HIP_OK(hipStreamWaitEvent(s.side, s.ev_ext_go, 0));
    set_iters_kernel<<<1, 64, 0, s.side>>>(s.d_ext_iter, iter, 1);
    ext();
    HIP_OK(hipEventRecord(s.ev_ext, s.side));
    s.side_pending |= 1;
    s.ext_launched = true;
  }
  HIP_OK(hipGraphLaunch(ge, s.stream));
  if (s.sharded && s.ar_per_graph_sweep > 0) s.ar_calls += (uint64_t)s.ar_per_graph_sweep * n;  // (RCCL: captured)
  return true;
}

static void eager_sweep(State& s, uint32_t iter, bool adapt) {
  if (s.graph_dirty) {  // state changed under the graphs: they are rebuilt after this sweep
    destroy_graph(s);
    s.graph_dirty = false;
    s.eager_streak = 0;
  }
  sweep(s, iter, adapt);
  s.eager_streak = adapt ? 0 : s.eager_streak + 1;
}

// part / nparts: this call's share of the sample -- Eta's factor columns h = part - 1 (mod
// nparts), everything else in part 0 (a run's last sample is unpacked by every worker, after the device
// is done: one worker took ~80 us of the 20-step run's tail)
static void unpack_record(const State& s, const double* slot, int k, int samples, hmsc_record* rec, int part = 0,
                          int nparts = 1) {
  const int K = s.K, nsl = s.nsl, nc = s.nc, nt = s.nt, NF = s.NF;
  const bool p0 = part == 0;
  const double* BL = slot;
  const double* Psi = BL + (size_t)K * nsl;
  const double* Delta = Psi + (size_t)NF * nsl;
  const double* Gamma = Delta + NF;
  const double* iV = Gamma + (size_t)nc * nt;
  const double* iS = iV + (size_t)nc * nc;
  const double* eta = iS + nsl;
  if (rec->Beta && p0)
    for (int j = 0; j < nsl; ++j)
      for (int c = 0; c < nc; ++c) rec->Beta[(size_t)k * nc * nsl + c + (size_t)nc * j] = BL[c + (size_t)K * j];
  if (rec->Gamma && p0) std::memcpy(rec->Gamma + (size_t)k * nc * nt, Gamma, sizeof(double) * nc * nt);
  if (rec->iV && p0) std::memcpy(rec->iV + (size_t)k * nc * nc, iV, sizeof(double) * nc * nc);
  if (rec->iSigma && p0) std::memcpy(rec->iSigma + (size_t)k * nsl, iS, sizeof(double) * nsl);
  for (int r = 0; r < s.nr; ++r) {
    const Level& L = s.lev[r];
    const int nf = L.nf, nfm = L.nfcap, lo = s.loff(r), fo = s.foff(r);
    if (rec->rec_nf && p0) rec->rec_nf[r * samples + k] = nf;
    if ((rec->Lambda[r] || rec->Psi[r]) && p0)
      for (int j = 0; j < nsl; ++j)
        for (int h = 0; h < nfm; ++h) {
          const size_t o = (size_t)k * nfm * nsl + h + (size_t)nfm * j;
          if (rec->Lambda[r]) rec->Lambda[r][o] = h < nf ? BL[lo + h + (size_t)K * j] : 0.0;
          if (rec->Psi[r]) rec->Psi[r][o] = h < nf ? Psi[fo + h + (size_t)NF * j] : 0.0;
        }
    for (int h = 0; h < nfm && p0; ++h) {
      if (rec->Delta[r]) rec->Delta[r][(size_t)k * nfm + h] = h < nf ? Delta[fo + h] : 1.0;
      if (rec->Alpha[r] && !L.spatial) rec->Alpha[r][(size_t)k * nfm + h] = 1;
    }
    if (rec->Eta[r])
      for (int h = (part + nparts - 1) % nparts; h < nfm; h += nparts) {  // (part 0 also has the rest)
        double* dst = rec->Eta[r] + (size_t)k * L.np * nfm + (size_t)L.np * h;
        if (h < nf)
          std::memcpy(dst, eta + (size_t)L.np * h, sizeof(double) * L.np);
        else
          std::memset(dst, 0, sizeof(double) * L.np);
      }
    eta += (size_t)L.np * nf;
  }
  if (!p0) return;
  if (rec->rho) rec->rho[k] = (int32_t)eta[0];  // packed after the Eta blocks (launch_record)
  const double* al = eta + 1;                   // then AlphaD of every spatial level
  for (int r = 0; r < s.nr; ++r) {
    const Level& L = s.lev[r];
    if (!L.spatial) continue;
    for (int h = 0; h < L.nfcap; ++h)
      if (rec->Alpha[r]) rec->Alpha[r][(size_t)k * L.nfcap + h] = h < L.nf ? (int32_t)al[h] : 1;
    al += L.nf;
  }
}

// First write to each page of sample k's slice of the caller's record arrays (zeros: every
// element of the slice is overwritten by unpack_record).  Fresh arrays (numpy zeros = untouched
// anonymous memory) fault on their first write, and that -- not the copy -- was most of an
// unpack (~100 us per 1.1 MB sample); an unpack worker does it for the sample it waits for,
// while the GPU is still producing it.
static void pretouch_record(const State& s, int k, const hmsc_record* rec) {
  constexpr size_t PG = 4096;
  auto touch = [&](void* base, size_t elem, size_t n) {
    if (!base || n == 0) return;
    char* p = (char*)base + (size_t)k * elem * n;
    const size_t bytes = elem * n;
    // first byte of the slice, then every page boundary inside it, then its last element
    volatile char* vp = p;
    vp[0] = 0;
    for (size_t o = PG - ((uintptr_t)p & (PG - 1)); o < bytes; o += PG) vp[o] = 0;
    vp[bytes - 1] = 0;
  };
  const size_t nc = s.nc, nsl = s.nsl;
  touch(rec->Beta, sizeof(double), nc * nsl);
  touch(rec->Gamma, sizeof(double), nc * s.nt);
  touch(rec->iV, sizeof(double), nc * nc);
  touch(rec->iSigma, sizeof(double), nsl);
  for (int r = 0; r < s.nr; ++r) {
    const size_t nfm = s.lev[r].nfcap;
    touch(rec->Eta[r], sizeof(double), (size_t)s.lev[r].np * nfm);
    touch(rec->Lambda[r], sizeof(double), nfm * nsl);
    touch(rec->Psi[r], sizeof(double), nfm * nsl);
  }
}

// Record-unpack workers kept for the life of a chain: starting W threads in every run() cost
// ~0.1 ms, a few percent of a 20-sweep run.  Between runs they sleep on a condition variable;
// a run hands them one job (worker w unpacks samples w, w + W, ...) and waits for all of them.
struct UnpackPool {
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv_job, cv_idle;
  std::function<void(int)> job;
  uint64_t gen = 0;
  int busy = 0;
  std::atomic<int> busy_a{0};  // busy, readable without the lock (wait_spin)
  bool quit = false;
  explicit UnpackPool(int W) {
    for (int w = 0; w < W; ++w) th.emplace_back([this, w] { loop(w); });
  }
  void loop(int w) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void(int)> f;
      {
        std::unique_lock<std::mutex> lk(m);
        cv_job.wait(lk, [&] { return quit || gen != seen; });
        if (quit) return;
        seen = gen;
        f = job;
      }
      f(w);  // never throws: the job records its own failure
      std::lock_guard<std::mutex> lk(m);
      busy_a.fetch_sub(1, std::memory_order_release);
      if (--busy == 0) cv_idle.notify_all();
    }
  }
  void start(std::function<void(int)> f) {
    std::lock_guard<std::mutex> lk(m);
    job = std::move(f);
    busy = (int)th.size();
    busy_a.store(busy, std::memory_order_relaxed);
    ++gen;
    cv_job.notify_all();
  }
  void wait_spin() {  // poll until every worker is through (then wait() returns at once)
    while (busy_a.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m);
    cv_idle.wait(lk, [&] { return busy == 0; });
    job = nullptr;  // drop the finished run's references
  }
  ~UnpackPool() {
    {
      std::lock_guard<std::mutex> lk(m);
      quit = true;
    }
    cv_job.notify_all();
    for (auto& t : th) t.join();
  }
};

static void run(State& s, int transient, int samples, int thin, const int* adaptNf, int iter0, int verbose,
                int chain, hmsc_record* rec) {
  const auto t_entry = std::chrono::steady_clock::now();
  DeviceGuard dg(s.device);
  HMSC_REQUIRE(thin >= 1 && samples >= 0 && transient >= 0, "bad transient/samples/thin");
  for (int r = 0; r < s.nr; ++r)
    HMSC_REQUIRE(adaptNf == nullptr || adaptNf[r] <= transient,
                 "transient parameter should be no less than any element of adaptNf parameter");
  const bool recording = rec != nullptr && samples > 0;
  // Recording: sample k is packed into device slot k % ring_slots (main stream), copied to the
  // pinned host slot (copy stream), after which a flag kernel bumps *copied_host to k + 1.
  // Host unpack threads poll that counter -- no HIP call off the launching thread, so nothing
  // contends with the sweep launches -- and unpack sample k into the caller's arrays (worker
  // k % W).  The launcher reuses slot k % ring_slots only after sample k - ring_slots is
  // unpacked, which also means its copy landed, so the device slot is free too.
  std::atomic<bool> stop{false}, worker_failed{false};
  std::string worker_err;
  std::mutex mu;                        // worker_err + cv_done
  std::condition_variable cv_done;
  std::unique_ptr<std::atomic<uint8_t>[]> done(new std::atomic<uint8_t>[std::max(1, samples)]);
  for (int k = 0; k < samples; ++k) done[k].store(0);
  int low = 0;  // every sample < low is unpacked (main thread only)
  std::atomic<int64_t> diag_unpack_ns{0};  // HMSC_DIAG_TIMING: time in unpack (all workers)
  std::atomic<int> last_parts{0};           // workers through their share of the last sample
  std::atomic<bool> last_touched{false};    // ... whose pages the launcher thread has touched
  int64_t diag_wait_ns = 0;                 // and the launcher's waits for a free ring slot
  volatile uint64_t* copied = s.copied_host;
  if (recording) *copied = 0;           // no copy is in flight between runs
  const char* w_env = getenv("HMSC_UNPACK_THREADS");
  const int W = recording ? std::max(1, std::min(w_env ? atoi(w_env) : 4,
                                                 std::max(1, (int)std::thread::hardware_concurrency() / 2)))
                          : 0;
  if (recording && (!s.unpack_pool || (int)s.unpack_pool->th.size() != W))
    s.unpack_pool = std::make_shared<UnpackPool>(W);
  UnpackPool* pool = recording ? s.unpack_pool.get() : nullptr;
  struct Joiner {  // an exception in the launch loop stops the workers before its locals go
    UnpackPool* p;
    std::atomic<bool>& stop;
    ~Joiner() {
      stop.store(true);
      if (p) p->wait();
    }
  } joiner{nullptr, stop};
  if (pool) {
    pool->start([&](int w) {
      try {
        // first touch of this worker's next samples' pages ahead of their data: a replay's
        // samples arrive together (one copy + flag per replay), so touching only the sample
        // being waited for left the later ones to fault inside their unpack
        constexpr int LOOKAHEAD = 4;
        int touched = w - W;
        // the run's last sample (W >= 2): every worker unpacks its share once it lands
        const int split = (W >= 2 && samples >= 1) ? samples - 1 : samples;
        for (int k = w; k < split; k += W) {
          while (touched + W < split && touched + W <= k + W * LOOKAHEAD) {
            touched += W;
            pretouch_record(s, touched, rec);
          }
          // spin (yielding) rather than sleep: a timed sleep oversleeps by the kernel's timer
          // slack (~50 us), which at the end of a short run is most of the unpack tail
          for (int spin = 0; __atomic_load_n(copied, __ATOMIC_ACQUIRE) <= (uint64_t)k; ++spin) {
            if (stop.load(std::memory_order_relaxed)) return;
            if (spin > (1 << 20)) std::this_thread::sleep_for(std::chrono::microseconds(20));
            else std::this_thread::yield();
          }
          const auto tu0 = std::chrono::steady_clock::now();
          unpack_record(s, s.host_rec + s.slot_doubles * (k % s.ring_slots), k, samples, rec);
          diag_unpack_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tu0).count();
          done[k].store(1, std::memory_order_release);
          {  // the launcher may be waiting for this host slot
            std::lock_guard<std::mutex> lk(mu);
          }
          cv_done.notify_one();
        }
        if (split < samples) {
          const int k = split;
          // (its pages are first touched by the launcher thread once the run is enqueued: a
          // worker's zero-write of a page could land after another worker's share)
          for (int spin = 0; __atomic_load_n(copied, __ATOMIC_ACQUIRE) <= (uint64_t)k ||
                             !last_touched.load(std::memory_order_acquire);
               ++spin) {
            if (stop.load(std::memory_order_relaxed)) return;
            if (spin > (1 << 20)) std::this_thread::sleep_for(std::chrono::microseconds(20));
            else std::this_thread::yield();
          }
          const auto tu0 = std::chrono::steady_clock::now();
          unpack_record(s, s.host_rec + s.slot_doubles * (k % s.ring_slots), k, samples, rec, w, W);
          diag_unpack_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tu0).count();
          if (last_parts.fetch_add(1, std::memory_order_acq_rel) == W - 1) {
            done[k].store(1, std::memory_order_release);
            {
              std::lock_guard<std::mutex> lk(mu);
            }
            cv_done.notify_one();
          }
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(mu);
        worker_err = e.what();
        worker_failed.store(true);
        cv_done.notify_all();
      }
    });
    joiner.p = pool;
  }
  const int total = transient + samples * thin;
  auto recorded = [&](int it) { return recording && it > transient && (it - transient) % thin == 0; };
  auto sample_of = [&](int it) { return (it - transient) / thin - 1; };
  // slot reuse: before sample k is packed, sample k - ring_slots must be unpacked (which
  // also means its copy landed, so the device slot is free as well)
  auto wait_slot = [&](int k) {
    const int need = k - s.ring_slots + 1;
    if (need <= 0) return;
    while (low < need && done[low].load(std::memory_order_acquire)) ++low;
    if (low < need) {
      const auto tw0 = std::chrono::steady_clock::now();
      struct Acc {
        std::chrono::steady_clock::time_point t0;
        int64_t& acc;
        ~Acc() { acc += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(); }
      } acc{tw0, diag_wait_ns};
      std::unique_lock<std::mutex> lk(mu);
      cv_done.wait(lk, [&] {
        while (low < need && done[low].load(std::memory_order_acquire)) ++low;
        return worker_failed.load() || low >= need;
      });
      if (worker_failed.load()) throw HmscError(-1, "record unpack: " + worker_err);
    }
  };
  auto copy_out = [&](int k) {
    const int slot = k % s.ring_slots;
    HIP_OK(hipMemcpyAsync(s.host_rec + s.slot_doubles * slot, s.ring + s.slot_doubles * slot,
                          sizeof(double) * s.slot_doubles, hipMemcpyDeviceToHost, s.copy_stream));
  };
  int max_adapt = 0;
  if (adaptNf)
    for (int r = 0; r < s.nr; ++r) max_adapt = std::max(max_adapt, adaptNf[r]);
  // the fused Gamma2 + BetaLambda flag holds the epoch of the last sweep that published: a
  // run's sweeps are distinct, but an earlier run may have ended on one of them
  // (the same for the tails epoch and the side chain's flags, graph sweeps' device-side joins)
  join_side(s);
  static_assert(2 + HMSC_MAX_LEVELS <= 56, "run_start_kernel: side flags");
  ++s.run_nonce;  // (kcopy: pack flags of an earlier run never match this run's)
  run_start_kernel<<<1, 64, 0, s.stream>>>(recording ? s.d_rec_desc : nullptr, iter0, transient, thin, samples,
                                           s.gbl_sync, s.crw_flag, s.side_sync, SIDE_SYNC_INTS, (int32_t)s.run_nonce);
  HIP_OK(hipGetLastError());
  const auto t_start = std::chrono::steady_clock::now();
  int n_replays = 0;
  for (int it = 1; it <= total;) {
    const int G = s.graph_sweeps;
    int n = 1;
    bool replayed = false;
    int kfirst = -1, klast = -1;
    if (it > max_adapt) {
      int ng = G;  // the run's remainder: its binary decomposition, largest graph first
      while (ng > 1 && it + ng - 1 > total) ng >>= 1;
      // a recorded run ends on single-sweep replays (..., 2, 1, 1): the samples of the last
      // replay are copied out only after it, so a small last replay shortens the copy tail
      // (not when that replay's graph copies each sample itself, kernel copies)
      if (recording && ng > 1 && it + ng - 1 == total && !s.long_tail && !(s.kcopy && ng <= s.kcopy_max)) ng >>= 1;
      // (optional) a short first replay: the graph launch submits the side stream's nodes only
      // after the main stream's, ~16 us of host time per sweep, so the side chain of a big
      // first replay's first sweep starts late (~0.35 ms at 32 sweeps) and the second sweep
      // waits for it; later replays are submitted while the previous one runs
      if (n_replays == 0 && s.first_replay > 0)
        while (ng > s.first_replay) ng >>= 1;
      for (int j = it; j < it + ng; ++j)
        if (recorded(j)) {
          if (kfirst < 0) kfirst = sample_of(j);
          klast = sample_of(j);
        }
      if (klast >= 0) wait_slot(klast);
      if (replay_sweeps(s, (uint32_t)(iter0 + it), klast >= 0, ng)) {
        replayed = true;
        ++n_replays;
        n = ng;
        const int pm = klast >= 0 ? s.gx_pack_mask[1][graph_level(ng)] : 0;
        if (klast >= 0 && pm > 0) {
          // kernel copies: each sample to the host ring as soon as its pack parts are in
          for (int k = kfirst; k <= klast; ++k) launch_rec_copy(s, k, pm);
          s.ext_launched = false;
        } else if (klast >= 0) {
          HIP_OK(hipEventRecord(s.ev_graph, s.stream));
          HIP_OK(hipStreamWaitEvent(s.copy_stream, s.ev_graph, 0));
          if (s.ext_launched) HIP_OK(hipStreamWaitEvent(s.copy_stream, s.ev_ext, 0));  // its record pack
          s.ext_launched = false;
          // the replay's samples in one copy per contiguous run of ring slots (at most two),
          // then one flag: a copy + flag per sample cost ~48 us of copy-engine and dispatch
          // time each (26 us of transfer), so a 32-sweep replay's copies backed up behind the
          // next replays and trailed the run's last sweep (rocprofv3 --memory-copy-trace)
          for (int k = kfirst; k <= klast;) {
            const int slot = k % s.ring_slots, nk = std::min(klast - k + 1, s.ring_slots - slot);
            HIP_OK(hipMemcpyAsync(s.host_rec + s.slot_doubles * slot, s.ring + s.slot_doubles * slot,
                                  sizeof(double) * s.slot_doubles * nk, hipMemcpyDeviceToHost, s.copy_stream));
            k += nk;
          }
          launch_copied_flag(s, (uint64_t)klast + 1);
        }
      }
    }
    if (!replayed) {
      eager_sweep(s, (uint32_t)(iter0 + it), it <= max_adapt);
      if (recorded(it)) {
        const int k = sample_of(it);
        wait_slot(k);
        record_after_sweep(s, s.ring + s.slot_doubles * (k % s.ring_slots));
        join_side(s);  // the copy below waits on the main stream only
        HIP_OK(hipEventRecord(s.ev_graph, s.stream));
        HIP_OK(hipStreamWaitEvent(s.copy_stream, s.ev_graph, 0));
        copy_out(k);
        launch_copied_flag(s, (uint64_t)k + 1);
      }
    }
    if (verbose > 0 && (it + n - 1) / verbose > (it - 1) / verbose) {
      HIP_OK(hipStreamSynchronize(s.stream));
      for (int j = it; j < it + n; ++j)
        if (j % verbose == 0)
          std::printf("[1] \"Chain %d, iteration %d of %d, (%s)\"\n", chain, j, total,
                      j > transient ? "sampling" : "transient");
      std::fflush(stdout);
    }
    it += n;
  }
  join_side(s);
  const auto t_enq = std::chrono::steady_clock::now();
  if (pool && W >= 2 && samples >= 1) {  // the last sample's pages, while the device runs
    pretouch_record(s, samples - 1, rec);
    last_touched.store(true, std::memory_order_release);
  }
  // HMSC_SPIN_WAIT=1: the run's end waited for by polling (the streams, the unpack workers)
  // instead of blocking waits, whose wake-up latency lands on every run's tail
  static const bool spin_wait = getenv_flag("HMSC_SPIN_WAIT");
  if (spin_wait) {
    for (hipStream_t q : {s.stream, s.copy_stream}) {
      hipError_t e;
      while ((e = hipStreamQuery(q)) == hipErrorNotReady) {
      }
      HIP_OK(e);
    }
  } else {
    HIP_OK(hipStreamSynchronize(s.stream));
    HIP_OK(hipStreamSynchronize(s.copy_stream));
  }
  const auto t_done = std::chrono::steady_clock::now();
  check_device_flags(s);
  if (recording) {
    if (spin_wait) pool->wait_spin();
    pool->wait();
    std::lock_guard<std::mutex> lk(mu);
    HMSC_REQUIRE(!worker_failed.load(), "record unpack: " + worker_err);
  }
  if (getenv("HMSC_DIAG_TIMING")) {  // host run-ahead diagnostic: enqueue time vs total
    const auto t_end = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr,
                 "[hmsc] run %d sweeps: setup %.3f ms, enqueued in %.3f ms, done in %.3f ms, unpacked + joined %.3f "
                 "ms later; unpack %.3f ms, slot waits %.3f ms\n",
                 total, ms(t_entry, t_start), ms(t_start, t_enq), ms(t_start, t_done), ms(t_done, t_end),
                 1e-6 * diag_unpack_ns.load(), 1e-6 * diag_wait_ns);
  }
}

}  // namespace hmsc

using namespace hmsc;

namespace hmsc {
void run_predict(const hmsc_predict_args* p, double* out);  // predict.hip
void post_omega(int device, int S, int ns, int nfmax, const int* nf, const double* Lambda, double* mean_cor,
                double* support, double* support_neg, double* mean_omega);  // post.hip
void post_vp(const hmsc_vp_args* v, double* out);
void post_ess(int device, int n, int p, const double* x, double* ess, int* order);
}

extern "C" {

const char* hmsc_last_error(void) { return g_last_error.c_str(); }

int hmsc_predict(const hmsc_predict_args* args, double* out) {
  return guarded([&] {
    HMSC_REQUIRE(args != nullptr && out != nullptr, "hmsc_predict: NULL argument");
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);  // it allocates (predict.hip)
    run_predict(args, out);
  });
}

int hmsc_post_omega(int32_t device, int32_t S, int32_t ns, int32_t nfmax, const int32_t* nf, const double* Lambda,
                    double* mean_cor, double* support, double* support_neg, double* mean_omega) {
  return guarded([&] {
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);  // it allocates
    DeviceGuard dg(device);
    post_omega(device, S, ns, nfmax, nf, Lambda, mean_cor, support, support_neg, mean_omega);
  });
}

int hmsc_variance_partitioning(const hmsc_vp_args* args, double* out) {
  return guarded([&] {
    HMSC_REQUIRE(args != nullptr, "hmsc_variance_partitioning: NULL argument");
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
    DeviceGuard dg(args->device);
    post_vp(args, out);
  });
}

int hmsc_effective_size(int32_t device, int32_t n, int32_t p, const double* x, double* ess, int32_t* order) {
  return guarded([&] {
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
    DeviceGuard dg(device);
    post_ess(device, n, p, x, ess, order);
  });
}

int hmsc_shard_range(int32_t ns, int32_t rank, int32_t nranks, int32_t* sp0, int32_t* nsl) {
  return guarded([&] {
    HMSC_REQUIRE(ns > 0 && nranks >= 1 && rank >= 0 && rank < nranks, "bad ns / rank / nranks");
    int a = 0, b = 0;
    HMSC_REQUIRE(shard_range(ns, rank, nranks, &a, &b) == 0, "species shard is empty: fewer than 4 species per rank");
    *sp0 = a;
    *nsl = b;
  });
}

int hmsc_dense_chol_solve(int32_t device, double* A, int32_t n, double* b, int32_t* info) {
  return guarded([&] {
    HMSC_REQUIRE(A != nullptr && n > 0 && info != nullptr, "hmsc_dense_chol_solve: bad arguments");
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
    DeviceGuard dg(device);
    DevBufs bufs;  // declared before the stream: the stream is synchronised before the frees
    OwnedStream os;
    const hipStream_t st = os.s;
    const size_t nn = (size_t)n * n;
    double* dA = bufs.alloc<double>(nn);
    double* db = bufs.alloc<double>(n);
    double* ws = bufs.alloc<double>(dense_ws_doubles(n));
    int* dinfo = bufs.alloc<int>(1);
    int* dsync = bufs.alloc<int>(DENSE_SYNC_INTS);  // the dense handshake block, zeroed
    HIP_OK(hipMemsetAsync(dinfo, 0, sizeof(int), st));
    HIP_OK(hipMemsetAsync(dsync, 0, DENSE_SYNC_INTS * sizeof(int), st));
    HIP_OK(hipMemcpyAsync(dA, A, nn * sizeof(double), hipMemcpyHostToDevice, st));
    if (b) HIP_OK(hipMemcpyAsync(db, b, (size_t)n * sizeof(double), hipMemcpyHostToDevice, st));
    dense_potrf_lower(st, dA, n, n, ws, dinfo, 0, dsync);
    if (b) {
      dense_trsv_lower(st, dA, n, n, db, 0, ws, 0, dsync);
      dense_trsv_lower(st, dA, n, n, db, 1, ws, 0, dsync);
      HIP_OK(hipMemcpyAsync(b, db, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipMemcpyAsync(A, dA, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(info, dinfo, sizeof(int), hipMemcpyDeviceToHost, st));
    int hs = 0;
    HIP_OK(hipMemcpyAsync(&hs, dsync + DENSE_SYNC_ERR, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (hs != 0)
      throw HmscError(-5, "internal: an in-launch handshake of the blocked dense solver timed out (error bits " +
                              std::to_string(hs) + "); the result is invalid");
  });
}

int hmsc_spatial_full_grid(int32_t device, int32_t np, int32_t sdim, const double* coords, const double* dist,
                           int32_t G, const double* alphas, double* iWg, double* RiWg, double* detWg) {
  return guarded([&] {
    HMSC_REQUIRE(np > 0 && G > 0 && alphas && iWg && RiWg && detWg && ((coords && sdim > 0) || dist),
                 "hmsc_spatial_full_grid: bad arguments");
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
    DeviceGuard dg(device);
    DevBufs bufs;
    OwnedStream os;
    const hipStream_t st = os.s;
    const size_t n2 = (size_t)np * np;
    double* geo = bufs.alloc<double>(coords ? (size_t)np * sdim : n2);
    copy_sync(geo, coords ? coords : dist, (coords ? (size_t)np * sdim : n2) * sizeof(double), hipMemcpyHostToDevice, st);
    double* dI = bufs.alloc<double>(n2 * G);
    double* dR = bufs.alloc<double>(n2 * G);
    double* dd = bufs.alloc<double>(G);
    int* flag = bufs.alloc<int>(1);
    HIP_OK(hipMemsetAsync(flag, 0, sizeof(int), st));
    HIP_OK(hipMemsetAsync(dI, 0, n2 * G * sizeof(double), st));
    HIP_OK(hipMemsetAsync(dR, 0, n2 * G * sizeof(double), st));
    spatial_full_grid(st, np, coords ? sdim : 0, coords ? geo : nullptr, coords ? nullptr : geo, alphas, G, dI, dR,
                      dd, flag);
    int bad = 0;  // every copy on the grid's own stream (ordered after its kernels)
    copy_sync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, st);
    copy_sync(iWg, dI, n2 * G * sizeof(double), hipMemcpyDeviceToHost, st);
    copy_sync(RiWg, dR, n2 * G * sizeof(double), hipMemcpyDeviceToHost, st);
    copy_sync(detWg, dd, G * sizeof(double), hipMemcpyDeviceToHost, st);
    HMSC_REQUIRE(bad == 0, "hmsc_spatial_full_grid: a grid matrix is not positive definite");
  });
}

int hmsc_device_count(int32_t* n) {
  return guarded([&] {
    int c = 0;
    HIP_OK(hipGetDeviceCount(&c));
    *n = c;
  });
}

int hmsc_comm_unique_id(void* out128) {
  return guarded([&] {
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    HMSC_REQUIRE(r == ncclSuccess, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
    std::memcpy(out128, &id, sizeof(id));
  });
}

int hmsc_create_sharded(const hmsc_model* model, uint64_t seed, int32_t device, uint32_t updater_mask,
                        int32_t rank, int32_t nranks, const void* comm_id, hmsc_state** out) {
  return guarded([&] {
    HMSC_REQUIRE(out != nullptr, "out is NULL");
    HMSC_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
    auto* h = new hmsc_state();
    try {
      build_state(h->s, model, seed, device, updater_mask, rank, nranks, comm_id);
    } catch (...) {
      free_state(h->s);
      delete h;
      throw;
    }
    *out = h;
  });
}

int hmsc_create_sharded_host(const hmsc_model* model, uint64_t seed, int32_t device, uint32_t updater_mask,
                             int32_t rank, int32_t nranks, hmsc_allreduce_fn fn, void* ctx, hmsc_state** out) {
  return guarded([&] {
    HMSC_REQUIRE(out != nullptr && fn != nullptr, "out / fn is NULL");
    HMSC_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
    auto* h = new hmsc_state();
    try {
      build_state(h->s, model, seed, device, updater_mask, rank, nranks, nullptr, fn, ctx);
    } catch (...) {
      free_state(h->s);
      delete h;
      throw;
    }
    *out = h;
  });
}

int hmsc_create(const hmsc_model* model, uint64_t seed, int32_t device, uint32_t updater_mask, hmsc_state** out) {
  return hmsc_create_sharded(model, seed, device, updater_mask, 0, 1, nullptr, out);
}

void hmsc_destroy(hmsc_state* h) {
  if (!h) return;
  try {
    free_state(h->s);
  } catch (...) {
  }
  delete h;
}

int hmsc_init_state(hmsc_state* h, const int32_t* nf0) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    if (nf0)
      for (int r = 0; r < s.nr; ++r) {
        HMSC_REQUIRE(nf0[r] >= 1 && nf0[r] <= s.lev[r].nfcap, "init: nf0 exceeds the level's factor capacity");
        s.lev[r].nf = nf0[r];
      }
    s.refresh_dims();
    HMSC_REQUIRE(s.K <= s.Kmax, "init: K = nc + sum(nf) exceeds the chain's capacity (<= 128)");
    join_side(s);
    clear_device_errors(s);
    launch_init(s);
    const double one = 1.0;  // rho = 1 (R/computeInitialParameters.R:226)
    HIP_OK(hipMemcpyAsync(s.rho, &one, sizeof(double), hipMemcpyHostToDevice, s.stream));
    s.graph_dirty = true;
    s.xeta_valid = false;
    s.g2s_valid = false;
    launch_update_z(s, 0, true);  // Z = updateZ(Y=hM$Y, ...) (R/computeInitialParameters.R:254)
    HIP_OK(hipStreamSynchronize(s.stream));
  });
}

int hmsc_init_z(hmsc_state* h) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    join_side(s);
    s.graph_dirty = true;
    s.g2s_valid = false;
    launch_update_z(s, 0, true);  // R/computeInitialParameters.R:254 (iter 0: the init stream)
    HIP_OK(hipStreamSynchronize(s.stream));
  });
}

int hmsc_set_state(hmsc_state* h, const hmsc_params* p) {
  return guarded([&] { set_state(h->s, p); });
}

int hmsc_get_state(hmsc_state* h, hmsc_params* p) {
  return guarded([&] { get_state(h->s, p); });
}

int hmsc_get_nf(hmsc_state* h, int32_t* nf) {
  return guarded([&] {
    for (int r = 0; r < h->s.nr; ++r) nf[r] = h->s.lev[r].nf;
  });
}

int hmsc_get_nf_cap(hmsc_state* h, int32_t* nfcap) {
  return guarded([&] {
    for (int r = 0; r < h->s.nr; ++r) nfcap[r] = h->s.lev[r].nfcap;
  });
}

int hmsc_sweep(hmsc_state* h, int32_t iter, int32_t adapt_nf) {
  return guarded([&] {
    DeviceGuard dg(h->s.device);
    eager_sweep(h->s, (uint32_t)iter, adapt_nf != 0);
  });
}

int hmsc_update(hmsc_state* h, uint32_t which, int32_t iter) {
  return guarded([&] {
    DeviceGuard dg(h->s.device);
    run_updater(h->s, which, (uint32_t)iter);
  });
}

int hmsc_set_noise_mode(hmsc_state* h, int32_t mode) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    s.noise_mode = mode & 1;
    s.graph_dirty = true;
    std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
    if ((mode & 2) && !s.dbg_prec) s.dbg_prec = dalloc<double>((size_t)s.nsl * s.Kmax * s.Kmax);
    if (!(mode & 2) && s.dbg_prec) {
      HIP_OK(hipStreamSynchronize(s.stream));
      HIP_OK(hipFree(s.dbg_prec));
      s.dbg_prec = nullptr;
    }
  });
}

int hmsc_run(hmsc_state* h, int32_t transient, int32_t samples, int32_t thin, const int32_t* adaptNf,
             int32_t iter0, hmsc_record* rec) {
  return guarded([&] { run(h->s, transient, samples, thin, adaptNf, iter0, 0, 1, rec); });
}

int hmsc_run_verbose(hmsc_state* h, int32_t transient, int32_t samples, int32_t thin, const int32_t* adaptNf,
                     int32_t iter0, int32_t verbose, int32_t chain, hmsc_record* rec) {
  return guarded([&] { run(h->s, transient, samples, thin, adaptNf, iter0, verbose, chain, rec); });
}

int hmsc_prepare_graphs(hmsc_state* h, int32_t iter, int32_t* built) {
  return guarded([&] {
    HMSC_REQUIRE(built != nullptr, "hmsc_prepare_graphs: built is NULL");
    State& s = h->s;
    DeviceGuard dg(s.device);
    *built = 0;
    if (!s.use_graph || s.prof) return;
    if (graphs_built(s) && s.graph_edge_free && live_chains(s.device) > 1) s.graph_dirty = true;
    if (graphs_built(s) && (s.graph_dirty || s.graph_K != s.K || s.graph_NF != s.NF)) destroy_graph(s);
    if (!graphs_built(s)) {
      if (s.graph_dirty) s.eager_streak = 0, s.graph_dirty = false;
      if (s.eager_streak < 1 || !build_sweep_graphs(s, (uint32_t)iter)) return;
    }
    // make the executable graphs device-resident now, not at their first launch
    for (auto& row : s.gx)
      for (hipGraphExec_t g : row)
        if (g) HIP_OK(hipGraphUpload(g, s.stream));
    for (auto& v : s.gseg)
      for (auto& sg : v) HIP_OK(hipGraphUpload(sg.g, s.stream));
    HIP_OK(hipStreamSynchronize(s.stream));
    *built = 1;
  });
}

int hmsc_sync(hmsc_state* h) {
  return guarded([&] {
    DeviceGuard dg(h->s.device);
    join_side(h->s);
    HIP_OK(hipStreamSynchronize(h->s.stream));
    HIP_OK(hipStreamSynchronize(h->s.copy_stream));
    check_device_flags(h->s);
  });
}

// Test hook: corrupt one of the chain's in-launch handshakes so the next launch that uses it
// must time out and report ("trsv_ticket": the sync-free solve's ticket starts at 1, so block 0
// is never solved; "chol_publish": the next fused panel step of the blocked Cholesky withholds
// its flag).
int hmsc_debug_poison(hmsc_state* h, const char* what) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    HMSC_REQUIRE(what != nullptr, "hmsc_debug_poison: what is NULL");
    join_side(s);
    HIP_OK(hipStreamSynchronize(s.stream));
    const std::string w(what);
    int v = 1, at = 0;
    if (w == "trsv_ticket") at = 0;
    else if (w == "chol_publish") at = DENSE_SYNC_TEST, v = HS_TEST_SKIP_PUBLISH;
    else throw HmscError(-1, "hmsc_debug_poison: unknown handshake " + w);
    copy_sync(s.trsv_sync + at, &v, sizeof(int), hipMemcpyHostToDevice, s.stream);
  });
}

int hmsc_debug_get(hmsc_state* h, const char* name, double* out, int64_t n) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    join_side(s);
    HIP_OK(hipStreamSynchronize(s.stream));
    const std::string nm(name);
    const double* src = nullptr;
    int64_t avail = 0;
    if (nm == "Z") src = s.Z, avail = (int64_t)s.ny * s.nsl;
    else if (nm == "XZ") flush_xz(s), src = s.XZ, avail = (int64_t)s.K * s.nsl;
    else if (nm == "G") flush_g(s), src = s.G, avail = (int64_t)s.Kmax * s.Kmax;
    else if (nm == "ZTr") src = s.ZTr, avail = (int64_t)s.ny * s.nt;
    else if (nm == "BL") src = s.BL, avail = (int64_t)s.K * s.nsl;
    else if (nm == "BL_prec") src = s.dbg_prec, avail = s.dbg_prec ? (int64_t)s.nsl * s.K * s.K : 0;
    else if (nm == "CR") src = s.CR, avail = (int64_t)s.Kmax * s.NFmax;
    else if (nm == "ZL") src = s.ZL_part, avail = (int64_t)s.zl_split * s.ny * s.NF;
    else if (nm == "stamps") {
      read_stamps(out, (int)n);
      return;
    } else if (nm == "kt") {  // raw live-timing words: per id, KT_SLOTS starts then KT_SLOTS ends (wall-clock ticks)
      HMSC_REQUIRE(s.d_kt != nullptr, "debug_get kt: kernel timing is off");
      const int64_t m = std::min<int64_t>(n, (int64_t)KT_N * 2 * KT_SLOTS);
      std::vector<unsigned long long> v((size_t)m);
      copy_sync(v.data(), s.d_kt, sizeof(unsigned long long) * m, hipMemcpyDeviceToHost, s.stream);
      for (int64_t i = 0; i < m; ++i) out[i] = (double)v[i];
      return;
    } else if (nm.rfind("spwork_doubles", 0) == 0) {  // a spatial level's workspace size (doubles)
      const int r = std::atoi(nm.c_str() + 14);
      HMSC_REQUIRE(r >= 0 && r < s.nr && s.lev[r].spatial && n >= 1, "debug_get: not a spatial level");
      out[0] = (double)spatial_work_doubles(s, r);
      return;
    } else if (nm.rfind("nngp_perm", 0) == 0 || nm.rfind("nngp_bw", 0) == 0) {  // NNGP factorization order
      const bool perm = nm.rfind("nngp_perm", 0) == 0;
      const int r = std::atoi(nm.c_str() + (perm ? 9 : 7));
      HMSC_REQUIRE(r >= 0 && r < s.nr && s.lev[r].nngp, "debug_get: not an NNGP level");
      const Level& L = s.lev[r];
      if (!perm) {
        HMSC_REQUIRE(n >= 1, "nngp_bw needs 1 slot");
        out[0] = L.nnBwUnits;
        return;
      }
      HMSC_REQUIRE(n >= L.np, "nngp_perm needs np slots");
      std::vector<int> pv(L.np);
      copy_sync(pv.data(), L.nnPerm, sizeof(int) * L.np, hipMemcpyDeviceToHost, s.stream);
      for (int i = 0; i < L.np; ++i) out[i] = pv[i];
      return;
    } else if (nm == "ar_calls") {  // sharded chain: [all-reduces so far, their doubles, per captured sweep, sharded]
      HMSC_REQUIRE(n >= 4, "ar_calls needs 4 slots");
      const double d[4] = {(double)s.ar_calls, (double)s.ar_doubles, (double)s.ar_per_graph_sweep, (double)s.sharded};
      std::memcpy(out, d, sizeof(d));
      return;
    } else if (nm == "graph") {
      HMSC_REQUIRE(n >= 4, "graph needs 4 slots");
      const int top = graph_level(s.graph_sweeps);
      const bool segs = host_segments(s);
      const double d[4] = {(double)(segs ? !s.gseg[0].empty() : s.gx[0][top] != nullptr),
                           (double)(segs ? !s.gseg[1].empty() : s.gx[1][top] != nullptr), (double)s.graph_sweeps,
                           (double)s.eager_streak};
      std::memcpy(out, d, sizeof(d));
      return;
    } else if (nm == "g2bl") {  // the last fused Gamma2 + BetaLambda launch: [partials trailing, grid size]
      HMSC_REQUIRE(n >= 2, "g2bl needs 2 slots");
      out[0] = (double)s.g2bl_last_tail;
      out[1] = (double)s.g2bl_last_nb;
      return;
    } else if (nm == "dims") {
      HMSC_REQUIRE(n >= 8, "dims needs 8 slots");
      const double d[8] = {(double)s.K, (double)s.NF, (double)s.Kmax, (double)s.NFmax, (double)s.nchunk,
                           (double)s.ntile_j, (double)s.zl_split, (double)s.zt_valid};
      std::memcpy(out, d, sizeof(d));
      return;
    } else
      throw HmscError(-1, "debug_get: unknown buffer " + nm);
    HMSC_REQUIRE(src != nullptr, "debug_get: buffer not allocated (enable with noise mode bit 2)");
    HMSC_REQUIRE(n <= avail, "debug_get: n exceeds buffer size");
    copy_sync(out, src, sizeof(double) * n, hipMemcpyDeviceToHost, s.stream);
  });
}

}  // extern "C"

extern "C" {

// Live per-kernel timing with HIP events on the chain's own stream (bench.py's
// roofline numbers): id 0 updateZ fused kernel, 1 updateEta Z-pass, 2 batched
// BetaLambda solve, 3 per-unit Eta solve, 4 whole sweep.
int hmsc_profile(hmsc_state* h, int32_t enable) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    HIP_OK(hipStreamSynchronize(s.stream));
    for (auto& v : s.prof_ev) {
      for (auto& e : v) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
      }
      v.clear();
    }
    s.prof = enable != 0;
  });
}

// Launch timing from inside the kernels (common.h kt_record), graph replays included.
int hmsc_kernel_timing(hmsc_state* h, int32_t enable) {
  return guarded([&] {
    State& s = h->s;
    DeviceGuard dg(s.device);
    join_side(s);
    HIP_OK(hipStreamSynchronize(s.stream));
    if (enable && !s.d_kt) {
      std::lock_guard<std::recursive_mutex> dev_lock(g_dev_mu);
      s.d_kt = dalloc<unsigned long long>((size_t)KT_N * 2 * KT_SLOTS);
    }
    if (enable)
      for (int id = 0; id < KT_N; ++id) {
        unsigned long long* b = s.d_kt + (size_t)id * 2 * KT_SLOTS;
        HIP_OK(hipMemsetAsync(b, 0xff, sizeof(unsigned long long) * KT_SLOTS, s.stream));  // starts: max
        HIP_OK(hipMemsetAsync(b + KT_SLOTS, 0, sizeof(unsigned long long) * KT_SLOTS, s.stream));
      }
    HIP_OK(hipStreamSynchronize(s.stream));
    if (s.kt_on != (enable != 0)) s.graph_dirty = true;  // the kernels' kt pointer changes
    s.kt_on = enable != 0;
  });
}

int hmsc_kernel_timing_get(hmsc_state* h, int32_t id, double* total_us, int32_t* count) {
  return guarded([&] {
    State& s = h->s;
    HMSC_REQUIRE(id >= 0 && id < KT_N, "kernel timing id out of range");
    *total_us = 0.0;
    *count = 0;
    if (!s.d_kt) return;
    DeviceGuard dg(s.device);
    join_side(s);
    HIP_OK(hipStreamSynchronize(s.stream));
    std::vector<unsigned long long> v((size_t)2 * KT_SLOTS);
    copy_sync(v.data(), s.d_kt + (size_t)id * 2 * KT_SLOTS, sizeof(unsigned long long) * v.size(),
                     hipMemcpyDeviceToHost);
    int khz = 0;
    HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, s.device));
    HMSC_REQUIRE(khz > 0, "wall clock rate unavailable");
    double ticks = 0.0;
    for (int i = 0; i < KT_SLOTS; ++i)
      if (v[KT_SLOTS + i] != 0 && v[i] != ~0ull && v[KT_SLOTS + i] >= v[i]) {
        ticks += (double)(v[KT_SLOTS + i] - v[i]);
        ++*count;
      }
    *total_us = ticks * 1e3 / khz;
  });
}

int hmsc_profile_get(hmsc_state* h, int32_t id, double* total_ms, int32_t* count) {
  return guarded([&] {
    State& s = h->s;
    HMSC_REQUIRE(id >= 0 && id < PROF_N, "profile id out of range");
    DeviceGuard dg(s.device);
    HIP_OK(hipStreamSynchronize(s.stream));
    double t = 0.0;
    for (auto& e : s.prof_ev[id]) {
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, e.first, e.second));
      t += ms;
    }
    *total_ms = t;
    *count = (int32_t)s.prof_ev[id].size();
  });
}

}  // extern "C"
