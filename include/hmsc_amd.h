/*
 * hmsc_amd.h — C ABI of the MI355X-native Gibbs sampler behind Hmsc's sampleMcmc().
 *
 * The reference (taddallas/HMSC, R package Hmsc 3.0-4) has no native code and no
 * FFI: its boundary is the R function sampleMcmc() (R/sampleMcmc.R:68-71) whose
 * per-chain body sampleChain() (R/sampleMcmc.R:155-327) runs the sweep loop
 * (:219-325) over R-level updaters.  Each entry point below names the reference
 * interface it replaces.  A maintainer binds them from R with the .Call shim in
 * INTEGRATION.md; this repository binds them with ctypes (hmsc_amd/_lib.py).
 *
 * Conventions
 *   - every matrix is column-major fp64 exactly as R stores it (no transposes);
 *   - Y carries R's NA as NaN; Pi is R's 1-based hM$Pi (stored as int32 here);
 *   - caller owns every input buffer; hmsc_create copies them to the device;
 *   - caller allocates every output buffer;
 *   - return 0 on success, <0 on error; hmsc_last_error() gives the message
 *     (thread-local); no C++ exception or longjmp crosses this boundary.
 */
#ifndef HMSC_AMD_H
#define HMSC_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HMSC_MAX_LEVELS 8

/* updater switches: R's updater=list(NAME=FALSE) (R/sampleMcmc.R:17,221-294) as a bitmask */
enum hmsc_updater {
  HMSC_UP_GAMMA2 = 1u << 0,       /* updateGamma2       R/updateGamma2.R:6      */
  HMSC_UP_GAMMAETA = 1u << 1,     /* updateGammaEta     R/updateGammaEta.R:7    */
  HMSC_UP_BETALAMBDA = 1u << 2,   /* updateBetaLambda   R/updateBetaLambda.R:8  */
  HMSC_UP_WRRR = 1u << 3,         /* updatewRRR         (out of scope)          */
  HMSC_UP_BETASEL = 1u << 4,      /* updateBetaSel      (out of scope)          */
  HMSC_UP_GAMMAV = 1u << 5,       /* updateGammaV       R/updateGammaV.R:4      */
  HMSC_UP_RHO = 1u << 6,          /* updateRho          R/updateRho.R:1         */
  HMSC_UP_LAMBDAPRIORS = 1u << 7, /* updateLambdaPriors R/updateLambdaPriors.R:3 */
  HMSC_UP_WRRRPRIORS = 1u << 8,   /* updatewRRRPriors   (out of scope)          */
  HMSC_UP_ETA = 1u << 9,          /* updateEta          R/updateEta.R:4         */
  HMSC_UP_ALPHA = 1u << 10,       /* updateAlpha        R/updateAlpha.R:3       */
  HMSC_UP_INVSIGMA = 1u << 11,    /* updateInvSigma     R/updateInvSigma.R:3    */
  HMSC_UP_Z = 1u << 12,           /* updateZ            R/updateZ.R:4           */
  HMSC_UP_ALL = 0x1FFFu
};

/* The hM fields consumed by the sampler (R/Hmsc.R:118-167 after construction and
 * setPriors defaults R/setPriors.Hmsc.R:28-77, R/setPriors.HmscRandomLevel.R:31-108).
 * Zero-initialise the struct and set struct_size = sizeof(hmsc_model) (HMSC_MODEL_SIZE):
 * hmsc_create refuses any other value, so a caller built against an older header (a shorter
 * struct) gets an error instead of having fields read past its end. */
typedef struct hmsc_model {
  int32_t struct_size;    /* sizeof(hmsc_model) of the header the caller was built with */
  int32_t ny, ns, nc, nt, nr;
  const double* Y;        /* ny*ns  hM$YScaled (NaN = NA)                      */
  const double* Yraw;     /* ny*ns  hM$Y (initial Z, R/computeInitialParameters.R:254); may equal Y */
  const double* X;        /* ny*nc  hM$XScaled                                 */
  const double* Tr;       /* ns*nt  hM$TrScaled                                */
  const int32_t* Pi;      /* ny*nr  hM$Pi, 1-based                             */
  const int32_t* np;      /* nr     hM$np                                      */
  const int32_t* distr;   /* ns*4   hM$distr (family, variance, link, -)       */
  const double* V0;       /* nc*nc  */
  double f0;
  const double* mGamma;   /* nc*nt  */
  const double* UGamma;   /* (nc*nt)^2 */
  const double* aSigma;   /* ns */
  const double* bSigma;   /* ns */
  /* per random level r < nr (hM$rL[[r]]) */
  const double* nu;
  const double* a1;
  const double* b1;
  const double* a2;
  const double* b2;
  const int32_t* nfMin;
  const int32_t* nfMax;
  const int32_t* sDim;    /* > 0: spatial level (see spatialMethod below); the number of
                           * coordinate columns when sCoord[r] is given             */
  const int32_t* xDim;    /* 0 for every level passed: a covariate-dependent level is passed
                           * expanded, see etaShare / xScale at the end */
  /* Phylogeny (hM$C; NULL = none).  The grid of R/computeDataParameters.R:19-39
   * (iQg/RQg/detQg over hM$rhopw) is taken in spectral form: the caller passes the
   * eigendecomposition of C (R: e <- eigen(hM$C, symmetric=TRUE); numpy: eigh), from which
   * every Q_g = rho_g C + (1-rho_g) I (or -rho_g iC + (1+rho_g) I for rho_g < 0) follows. */
  const double* C;        /* ns*ns (only tested for != NULL)                  */
  int32_t nrho;           /* nrow(hM$rhopw)                                    */
  const double* rhopw;    /* nrho*2 column-major: grid value, prior weight     */
  const double* C_vectors;/* ns*ns eigenvectors of C, column-major             */
  const double* C_values; /* ns    eigenvalues of C (> 0)                      */
  /* Spatial levels (rL$sDim > 0): the alphapw grid of R/computeDataParameters.R:47-196,
   * per level r (entries of non-spatial levels ignored / NULL), as the dense prior
   * precision of each grid point.  iWg, RiWg are np*np*nalpha column-major (R's
   * [np, np, alphaN] arrays) with RiWg' RiWg = iWg, detWg nalpha = log det W.  RiWg is
   * upper triangular, except for NNGP (R's lower-triangular factor) and GPP (lower).
   *   Full: computeDataParameters' iWg / RiWg / detWg as they are (:53-81).
   *   NNGP: not through these arrays -- sCoord and nNeighbours below (sparse Vecchia form).
   *   GPP:  iWg = diag(idDg[,g]) - idDW12g[,,g] iFg[,,g] t(idDW12g[,,g]) = W^-1, passed as
   *         RiWg = solve(t(chol(W))) (lower) with W = D + W12 iW22 t(W12), iWg = t(RiWg) RiWg,
   *         detWg = detDg (:138-194; the precision R/updateEta.R:148-196 samples from).
   * NNGP and GPP levels need np == ny (R/updateEta.R:140,165 build Diagonal(ny)). */
  const int32_t* spatialMethod;              /* nr: 0 none, 1 Full, 2 NNGP, 3 GPP        */
  const int32_t* nalpha;                     /* nr: nrow(rL$alphapw)                     */
  const double* alphapw[HMSC_MAX_LEVELS];    /* nalpha*2: grid value, prior weight      */
  const double* iWg[HMSC_MAX_LEVELS];      /* Full (host grid) only; NNGP: see sCoord */
  const double* RiWg[HMSC_MAX_LEVELS];
  const double* detWg[HMSC_MAX_LEVELS];
  /* 'Full' levels may leave iWg / RiWg / detWg NULL and hand over the level's geometry
   * instead -- the coordinates hM$rL[[r]]$s of its units in unit order (np x sDim[r],
   * column-major) or their distance matrix (np x np) --: the device then evaluates the grid
   * itself (dist(), exp(-d/alpha), chol, inverse on the matrix cores), storing
   * RiWg = chol(W_g)^-1 (lower; RiWg' RiWg = iWg as before).  At np = 5000 this is the
   * path that fits: two 20 GB grids are built in HBM without a host copy. */
  const double* sCoord[HMSC_MAX_LEVELS];
  const double* distMat[HMSC_MAX_LEVELS];
  /* 'GPP' levels may instead (iWg / RiWg / detWg NULL) hand over computeDataParameters'
   * predictive-process grid as R keeps it (R/computeDataParameters.R:138-194): nKnots[r]
   * knots, idDg (np x nalpha), idDW12g (np x nK x nalpha), Fg and iFg (nK x nK x nalpha),
   * detDg (nalpha), all column-major.  updateEta then samples R's low-rank form
   * (R/updateEta.R:148-196: per-unit nf x nf blocks and one (nK nf)^2 factorization, no
   * np^2 array anywhere) and updateAlpha evaluates R's GPP statistic (R/updateAlpha.R:35-75). */
  const int32_t* nKnots;                     /* nr (entries of non-GPP levels ignored)  */
  const double* idDg[HMSC_MAX_LEVELS];
  const double* idDW12g[HMSC_MAX_LEVELS];
  const double* Fg[HMSC_MAX_LEVELS];
  const double* iFg[HMSC_MAX_LEVELS];
  const double* detDg[HMSC_MAX_LEVELS];
  /* 'NNGP' levels (spatialMethod 2) hand over the coordinates of their units (sCoord[r], unit
   * order) and rL$nNeighbours (nNeighbours[r]; R's default 10): the library finds the nearest
   * earlier neighbours (FNN::get.knn restated), evaluates the Vecchia factor of every alphapw
   * grid point (R/computeDataParameters.R:82-136) and samples in that sparse form (np nNeighbours
   * numbers per grid point; updateEta factors the band of the precision in reverse Cuthill-McKee
   * order).  NNGP levels never take iWg / RiWg. */
  const int32_t* nNeighbours;                /* nr (entries of non-NNGP levels ignored) */
  /* Covariate-dependent levels (HmscRandomLevel(xData=...), rL$xDim = ncr > 0): R's
   * LRan = sum_k (Eta[Pi,] * x[dfPi, k]) %*% Lambda[,,k] (R/updateZ.R:24-29) is passed as ncr
   * consecutive levels r0 .. r0+ncr-1 that share the units (same np, Pi), nf and Eta:
   * etaShare[r] = r0 for each of them (the level whose Eta they use; r itself, or a negative
   * value, for an ordinary level; NULL: none shared) and xScale[r] = column k of rL$x in unit
   * order (np doubles), so level r0+k's XEta columns are Eta[Pi,] * x[Pi, k] and its Lambda,
   * Psi and Delta are R's Lambda[,,k], Psi[,,k] and Delta[,k] with priors nu[k], a1[k], b1[k],
   * a2[k], b2[k] (R/updateBetaLambda.R:22-53, R/updateLambdaPriors.R:34-48).  updateEta draws
   * the shared Eta once per unit from lambdaLocal = sum_k x[q, k] Lambda[,,k]
   * (R/updateEta.R:93-108) and updateNf adds or drops a factor of all ncr levels together
   * (R/updateNf.R).  Not with spatial levels, updateGammaEta or species sharding. */
  const int32_t* etaShare;                   /* nr, or NULL                              */
  const double* xScale[HMSC_MAX_LEVELS];     /* np[r] each, or NULL                      */
} hmsc_model;

#define HMSC_MODEL_SIZE ((int32_t)sizeof(hmsc_model))

/* Sampler state = R's parList (R/computeInitialParameters.R:256-270) with iV in
 * place of V and iSigma in place of sigma, as sampleChain keeps them
 * (R/sampleMcmc.R:161-177).  Per-level arrays are indexed [r]; Eta[r] is
 * np[r]*nf[r], Lambda/Psi[r] nf[r]*ns, Delta/Alpha[r] nf[r] (Alpha 1-based grid index). */
typedef struct hmsc_params {
  double* Gamma;          /* nc*nt */
  double* iV;             /* nc*nc */
  double* Beta;           /* nc*ns */
  double* iSigma;         /* ns    */
  double* Z;              /* ny*ns (may be NULL) */
  int32_t rho;            /* 1-based */
  int32_t nf[HMSC_MAX_LEVELS];
  double* Eta[HMSC_MAX_LEVELS];
  double* Lambda[HMSC_MAX_LEVELS];
  double* Psi[HMSC_MAX_LEVELS];
  double* Delta[HMSC_MAX_LEVELS];
  int32_t* Alpha[HMSC_MAX_LEVELS];
} hmsc_params;

/* Recording buffers for hmsc_run: caller-allocated, `samples` slots each.  The
 * fields are the raw (scaled-X) state; the host applies combineParameters
 * (R/combineParameters.R:1-58) afterwards.  Eta/Lambda/Psi/Delta/Alpha slots are
 * padded to nfcap[r] (hmsc_get_nf_cap: min(nfMax[r], the K <= 64 limit)); rec_nf[r*samples+k]
 * gives the live nf of sample k. */
typedef struct hmsc_record {
  double* Beta;           /* samples*nc*ns */
  double* Gamma;          /* samples*nc*nt */
  double* iV;             /* samples*nc*nc */
  double* iSigma;         /* samples*ns    */
  int32_t* rho;           /* samples       */
  double* Eta[HMSC_MAX_LEVELS];     /* samples*np[r]*nfcap[r]  */
  double* Lambda[HMSC_MAX_LEVELS];  /* samples*nfcap[r]*ns     */
  double* Psi[HMSC_MAX_LEVELS];     /* samples*nfcap[r]*ns     */
  double* Delta[HMSC_MAX_LEVELS];   /* samples*nfcap[r]        */
  int32_t* Alpha[HMSC_MAX_LEVELS];  /* samples*nfcap[r]        */
  int32_t* rec_nf;                  /* nr*samples              */
} hmsc_record;

typedef struct hmsc_state hmsc_state;

/* Thread-local description of the last error. */
const char* hmsc_last_error(void);

/* Number of visible MI355X devices. */
int hmsc_device_count(int32_t* n);

/* Create one chain's device state: copies the model, allocates HBM for the state
 * at nfcap (hmsc_get_nf_cap; work buffers of the dense updaters follow the nf in use), keys Philox by `seed` (R: set.seed(initSeed[chain]), R/sampleMcmc.R:158).
 * Replaces the per-chain setup of sampleChain, R/sampleMcmc.R:155-216. */
int hmsc_create(const hmsc_model* model, uint64_t seed, int32_t device, uint32_t updater_mask,
                hmsc_state** out);

/* Species-sharded single chain: this rank owns species
 * [sp_begin, sp_end) of the model passed in full; `comm_id` is the 128-byte RCCL
 * unique id from hmsc_comm_unique_id() broadcast by rank 0 (NULL when nranks==1). */
int hmsc_create_sharded(const hmsc_model* model, uint64_t seed, int32_t device,
                        uint32_t updater_mask, int32_t rank, int32_t nranks,
                        const void* comm_id, hmsc_state** out);
int hmsc_comm_unique_id(void* out128);

/* The same species-sharded chain with a host transport in place of RCCL: every cross-shard
 * fp64 sum calls fn(buf, n, ctx), which must replace the n doubles at buf (host memory) by
 * their sum over all ranks and return 0.  For hosts without a device-to-device fabric, and
 * for exercising the sharded path on one GPU (several ranks, one device). */
typedef int (*hmsc_allreduce_fn)(double* buf, int64_t n, void* ctx);
int hmsc_create_sharded_host(const hmsc_model* model, uint64_t seed, int32_t device,
                             uint32_t updater_mask, int32_t rank, int32_t nranks,
                             hmsc_allreduce_fn fn, void* ctx, hmsc_state** out);
/* The species block [sp0, sp0 + nsl) rank `rank` of `nranks` owns in hmsc_create_sharded:
 * whole species quads (updateZ's Philox species quads), the ceil(ns/4) quads spread evenly,
 * rank r owning quads [floor(r Q/nranks), floor((r+1) Q/nranks)); an error if that block is
 * empty (fewer quads than ranks).  No reference counterpart (species sharding is new). */
int hmsc_shard_range(int32_t ns, int32_t rank, int32_t nranks, int32_t* sp0, int32_t* nsl);

void hmsc_destroy(hmsc_state* s);

/* computeInitialParameters(hM, initPar=NULL) on the device, including the initial
 * updateZ (R/computeInitialParameters.R:17-273). nf0[r] = starting nf (nfMin). */
int hmsc_init_state(hmsc_state* s, const int32_t* nf0);

/* initPar / resume: overwrite state (R/computeInitialParameters.R:82-227). */
int hmsc_set_state(hmsc_state* s, const hmsc_params* p);
int hmsc_get_state(hmsc_state* s, hmsc_params* p);
int hmsc_get_nf(hmsc_state* s, int32_t* nf);
/* nfcap[r]: the factors level r's buffers and record slots hold, min(nfMax_r, 64 - nc - the
 * other levels' nfMin) (K = nc + sum(nf) <= 64 in this build).  Below nfMax_r (R's default
 * nfMax = ns for many species) the run fails with -6 only if updateNf must grow the level
 * past it.  hmsc_record's per-level arrays are strided by nfcap, not nfMax. */
int hmsc_get_nf_cap(hmsc_state* s, int32_t* nfcap);

/* The closing step of computeInitialParameters: Z = updateZ(Y = hM$Y, Z = LFix + LRan, ...)
 * at the CURRENT state (R/computeInitialParameters.R:229-254) -- after hmsc_set_state has
 * applied an initPar (or initPar = "fixed effects", :52-79), as the reference draws Z last. */
int hmsc_init_z(hmsc_state* s);

/* One Gibbs sweep in the reference block order, R/sampleMcmc.R:219-306.
 * `iter` is the 1-based sweep number (Philox counter word 3 and updateNf's iter). */
int hmsc_sweep(hmsc_state* s, int32_t iter, int32_t adapt_nf);

/* A single updater (per-updater tests; R's tests call updaters directly,
 * tests/testthat/test-sampling.R). `which` is one hmsc_updater bit. */
int hmsc_update(hmsc_state* s, uint32_t which, int32_t iter);

/* noise_mode 1: every Gaussian innovation is zero, so Gaussian blocks return their
 * conditional means (moment-parity tests); 0: normal sampling. */
int hmsc_set_noise_mode(hmsc_state* s, int32_t mode);

/* The sweep loop with recording: for iter in 1..transient+samples*thin, record when
 * iter>transient and (iter-transient)%%thin==0 (R/sampleMcmc.R:219-315).
 * adaptNf[r] = hM adaptNf.  `rec` may be NULL (no recording). */
int hmsc_run(hmsc_state* s, int32_t transient, int32_t samples, int32_t thin,
             const int32_t* adaptNf, int32_t iter0, hmsc_record* rec);

/* hmsc_run with R's progress print every `verbose` sweeps
 * ("Chain %d, iteration %d of %d, (%s)", R/sampleMcmc.R:317-324). */
int hmsc_run_verbose(hmsc_state* s, int32_t transient, int32_t samples, int32_t thin,
                     const int32_t* adaptNf, int32_t iter0, int32_t verbose, int32_t chain,
                     hmsc_record* rec);

/* Live kernel timing with HIP events on the chain's stream (bench / roofline):
 * id 0 = fused updateZ kernel, 1 = updateEta Z-pass, 2 = batched BetaLambda solve,
 * 3 = per-unit Eta solve, 4 = whole sweep, 5 = spatial updateEta (dense system), 6 = its
 * blocked Cholesky, 7 = updateAlpha.  hmsc_profile(s,1) clears and enables. */
int hmsc_profile(hmsc_state* s, int32_t enable);
int hmsc_profile_get(hmsc_state* s, int32_t id, double* total_ms, int32_t* count);

/* Live launch timing measured inside the kernels (bench.py's roofline figure): every
 * workgroup reads the constant-rate wall clock when it starts and finishes; a launch's
 * duration is its last finish minus its first start, kept per sweep (graph replays
 * included; up to 8192 sweeps per window).  id 0 = updateZ kernel, 1 = fused updateEta
 * kernel, 2 = BetaLambda wave kernel.  hmsc_kernel_timing(s,1) clears and enables (0
 * disables); _get returns the summed duration (us) and the number of timed launches.
 * No reference counterpart: instrumentation of this port. */
int hmsc_kernel_timing(hmsc_state* s, int32_t enable);
int hmsc_kernel_timing_get(hmsc_state* s, int32_t id, double* total_us, int32_t* count);

/* ---- post-sampling statistics on the device ----
 * Reductions over posterior samples that return only their summaries; every sum is in a
 * fixed order, so results repeat bit for bit. */

/* computeAssociations (R/computeAssociations.R) and getPostEstimate(hM, "Omega")
 * (R/getPostEstimate.R) for one random level: Lambda holds S samples of nfmax x ns
 * (column-major each; factors h >= nf[s] ignored).  Outputs ns x ns: the mean of
 * cov2cor(Lambda_s' Lambda_s), its support mean(> 0), and for Omega_s = Lambda_s' Lambda_s the
 * posterior mean and mean(Omega_s < 0). */
int hmsc_post_omega(int32_t device, int32_t S, int32_t ns, int32_t nfmax, const int32_t* nf,
                    const double* Lambda, double* mean_cor, double* support, double* support_neg,
                    double* mean_omega);

/* computeVariancePartitioning (R/computeVariancePartitioning.R:37-204; X a matrix): the
 * caller passes the S samples the reference loops over (its quirk: `for (i in 1:hM$samples)`
 * over the pooled list, i.e. the first chain when nChains > 1), cM = cov(hM$X), and the group
 * of every covariate (1-based).  out (nc + 1 + ns (1 + nr + ngroups) doubles):
 * R2T.Beta (nc) | R2T.Y | fixed (ns) | random (nr x ns) | fixedsplit (ngroups x ns),
 * all already averaged over the samples; vals = fixed * fixedsplit and random follow on the host. */
typedef struct hmsc_vp_args {
  int32_t device, ny, ns, nc, nt, S, ngroups, nr;
  const int32_t* group;     /* nc */
  const double* X;          /* ny x nc  hM$X */
  const double* Tr;         /* ns x nt  hM$Tr */
  const double* cM;         /* nc x nc  cov(hM$X) */
  const double* Beta;       /* S x (nc x ns) */
  const double* Gamma;      /* S x (nc x nt) */
  const int32_t* nf;        /* nr x S: factors of level r in sample s at [r S + s] */
  int32_t nfmax[HMSC_MAX_LEVELS];
  const double* Lambda[HMSC_MAX_LEVELS];  /* S x (nfmax_r x ns) */
} hmsc_vp_args;
int hmsc_variance_partitioning(const hmsc_vp_args* args, double* out);

/* coda::effectiveSize of each column of x (n x p, column-major; one chain): n var / spec0
 * with spectrum0.ar (AR order by AIC up to min(n - 1, 10 log10 n), Yule-Walker by
 * Levinson-Durbin).  ess[p]; order[p] (may be NULL) the chosen AR orders. */
int hmsc_effective_size(int32_t device, int32_t n, int32_t p, const double* x, double* ess, int32_t* order);

/* Wait for all device work of this chain; fails (-1 not positive definite, -5 a timed-out
 * in-launch handshake) if any of it raised a device error flag. */
int hmsc_sync(hmsc_state* s);

/* Capture (without running) the steady-state sweep graphs that hmsc_run replays, so a
 * caller that times hmsc_run (bench.py) does not pay for stream capture and
 * hipGraphInstantiate inside its timed region.  `iter` is the next sweep index the caller
 * will run (the Philox counters of a replay are set per launch, so any value works).
 * *built = 1 when the graphs exist afterwards; 0 when the chain is not in a steady state
 * yet (no eager sweep since the last init / set_state / updateNf repack), is sharded, or
 * graphs are disabled (HMSC_NO_GRAPH, profiling) -- hmsc_run then captures on its own.
 * No reference counterpart: the R loop has no launch overhead to amortise. */
int hmsc_prepare_graphs(hmsc_state* s, int32_t iter, int32_t* built);

/* The blocked device Cholesky (dense.hip) on one host matrix, for tests: A (n x n,
 * column-major, lower triangle read) is overwritten by L (A = L L^T; the strict upper
 * triangle is scratch), b (may be NULL) by A^-1 b through L^-T L^-1; *info = 1 if A is not
 * positive definite.  Instrumentation of this port, no reference counterpart. */
int hmsc_dense_chol_solve(int32_t device, double* A, int32_t n, double* b, int32_t* info);

/* computeDataParameters' 'Full' grid (R/computeDataParameters.R:53-81) on the device, for
 * np units given by coordinates (np x sdim, column-major) or a distance matrix (np x np;
 * coords NULL) over the G grid values alphas: iWg, RiWg (np*np*G) and detWg (G) exactly as
 * hmsc_model takes them, RiWg = chol(W_g)^-1 lower triangular.  This is what hmsc_create
 * runs for a 'Full' level passed by sCoord / distMat. */
int hmsc_spatial_full_grid(int32_t device, int32_t np, int32_t sdim, const double* coords, const double* dist,
                           int32_t G, const double* alphas, double* iWg, double* RiWg, double* detWg);

/* Copy a named internal device buffer (fp64) for tests / profiling:
 * "Z", "E", "XEtaTZ", "Gram", "ZTr", "BL", "BL_prec" ... ; n = element count. */
int hmsc_debug_get(hmsc_state* s, const char* name, double* out, int64_t n);

/* Test hook: corrupt one in-launch handshake of this chain so the next launch that uses it
 * times out (about 1 s) and reports: "trsv_ticket" (the sync-free triangular solve's block
 * ticket) or "chol_publish" (the blocked Cholesky's fused panel flag, withheld once).  The next
 * hmsc_run / hmsc_sync / hmsc_get_state then fails with code -5 ("... handshake timed out").
 * Instrumentation of this port, no reference counterpart. */
int hmsc_debug_poison(hmsc_state* s, const char* what);

/* predict.Hmsc (R/predict.R:1-231) for a pooled posterior: every sample's
 * L = X Beta + sum_r Eta_r[Pi_r,] Lambda_r, then expected values (pnorm / exp(L + sigma/2) / L)
 * or draws (1[L + sqrt(sigma) e > 0] / rpois / L + sqrt(sigma) e), then the YScalePar
 * back-transform.  Replaces the per-sample loop of R/predict.R:143-229; the caller (the R
 * wrapper) keeps predictLatentFactor (R/predict.R:120-129) and passes the per-sample Eta rows
 * of the prediction units.  Arrays are sample-major stacks of R's column-major matrices. */
typedef struct hmsc_predict_args {
  int32_t ny, ns, nc, nr, nsamples;
  int32_t expected;       /* R's `expected` */
  uint64_t seed;          /* Philox key of the draws (expected = 0) */
  int32_t device;
  const double* X;        /* ny*nc  (unscaled X, as post holds un-scaled Beta) */
  const double* Beta;     /* nsamples*nc*ns */
  const double* sigma;    /* nsamples*ns */
  const int32_t* family;  /* ns: hM$distr[,1] */
  const double* YScalePar;/* 2*ns */
  const int32_t* Pi;      /* ny*nr, 1-based rows of the per-level Eta */
  const int32_t* np;      /* nr */
  const int32_t* nf;      /* nr */
  const double* Eta[HMSC_MAX_LEVELS];     /* nsamples*np[r]*nf[r] */
  const double* Lambda[HMSC_MAX_LEVELS];  /* nsamples*nf[r]*ns */
} hmsc_predict_args;

/* out: nsamples*ny*ns (pred[[s]] column-major, sample-major stack) */
int hmsc_predict(const hmsc_predict_args* args, double* out);

#ifdef __cplusplus
}
#endif
#endif /* HMSC_AMD_H */
