// updateZ launcher (R/updateZ.R:4-94): the fused z kernel of z_kernel.h and its slab
// reductions.  Its own translation unit: it is compiled with MachineLICM off (build.py), so
// the ~60 polynomial constants of the inlined truncated-normal draws are materialised where
// they are used inside the site loop instead of being hoisted into (and spilled from) the
// register file.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "rng.h"
#include "state.h"
#include "z_kernel.h"

namespace hmsc {

PackArgs record_pack_args(State& s, int part);  // kernels.hip

// Z Tr is only consumed with NA (updateGamma2 forms X^T Z Tr from XZ otherwise, and a
// sharded chain all-reduces that), so the no-NA kernels skip the ZTr contraction
template <bool HAS_NA>
constexpr int z_mode() { return HAS_NA ? Z_ALL : (Z_ALL & ~8); }

template <bool DRAW, bool HAS_NA, bool POIS, bool NORMAL>
static void z_dispatch_k(const State& s, dim3 grid, size_t smem, const ZArgs& a) {
  constexpr int M = z_mode<HAS_NA>();
  switch (z_nkb(s.K)) {
    case 1: z_wave_kernel<DRAW, HAS_NA, 1, M, POIS, NORMAL><<<grid, 256, smem, s.stream>>>(a); break;
    case 2: z_wave_kernel<DRAW, HAS_NA, 2, M, POIS, NORMAL><<<grid, 256, smem, s.stream>>>(a); break;
    case 3: z_wave_kernel<DRAW, HAS_NA, 3, M, POIS, NORMAL><<<grid, 256, smem, s.stream>>>(a); break;
    case 4: z_wave_kernel<DRAW, HAS_NA, 4, M, POIS, NORMAL><<<grid, 256, smem, s.stream>>>(a); break;
    default: z_wave_kernel<DRAW, HAS_NA, 8, M, POIS, NORMAL><<<grid, 256, smem, s.stream>>>(a); break;
  }
}

template <bool DRAW, bool HAS_NA, bool POIS = false>
static void z_dispatch(const State& s, dim3 grid, size_t smem, const ZArgs& a) {
  if (!DRAW || POIS || s.any_normal)
    z_dispatch_k<DRAW, HAS_NA, POIS, true>(s, grid, smem, a);
  else
    z_dispatch_k<DRAW, HAS_NA, POIS, false>(s, grid, smem, a);
}

template <bool HAS_NA>
static int z_occupancy(int nkb, size_t smem) {
  int nb = 0;
  switch (nkb) {
    case 1: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, z_wave_kernel<true, HAS_NA, 1, z_mode<HAS_NA>()>, 256, smem)); break;
    case 2: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, z_wave_kernel<true, HAS_NA, 2, z_mode<HAS_NA>()>, 256, smem)); break;
    case 3: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, z_wave_kernel<true, HAS_NA, 3, z_mode<HAS_NA>()>, 256, smem)); break;
    case 4: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, z_wave_kernel<true, HAS_NA, 4, z_mode<HAS_NA>()>, 256, smem)); break;
    default: HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, z_wave_kernel<true, HAS_NA, 8, z_mode<HAS_NA>()>, 256, smem)); break;
  }
  return nb;
}

int z_xeta_cols_for(int Kmax) { return z_xeta_cols(Kmax); }

// Workgroups of the drawing z kernel resident on the whole device at once (occupancy x CUs):
// the site-chunk count is sized so the (chunk x species-block) grid fills exactly one round.
int z_resident_slots(const State& s) {
  const size_t smem = z_smem_bytes(s.Kmax, s.nt);
  const int nkb = z_nkb(s.Kmax);
  int ncu = 0;
  const int nb = s.has_na ? z_occupancy<true>(nkb, smem) : z_occupancy<false>(nkb, smem);
  HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s.device));
  return std::max(1, nb) * std::max(1, ncu);
}

static void run_z_fused(State& s, bool draw, uint32_t iter, bool use_raw_y) {
  HMSC_REQUIRE(s.K <= KMAX_Z, "updateZ: K = nc + sum(nf) must be <= 128 in this build");
  HMSC_REQUIRE((s.sp0 & 1) == 0, "updateZ: species shards must start at an even species (Philox pairs)");
  if (!s.xeta_valid) launch_xeta(s);
  ZArgs a{};
  a.XEta = s.XEta;
  a.ny = s.ny;
  a.K = s.K;
  a.ns_loc = s.nsl;
  a.sp0 = s.sp0;
  a.nt = s.nt;
  const int n_tiles = (s.ny + ZT_I - 1) / ZT_I;
  a.tiles_per_chunk = (n_tiles + s.nchunk - 1) / s.nchunk;
  const int nchunk = (n_tiles + a.tiles_per_chunk - 1) / a.tiles_per_chunk;
  a.BL = s.BL;
  a.iSigma = s.iSigma;
  a.Ycode = s.Ycode;
  a.Ybits = s.Ybits;
  a.logtab = s.logtab;
  a.ztab = s.logtab + ZLOG_W * ZLOG_N;
  a.Yval = use_raw_y ? s.Yraw : s.Yval;
  a.fam = s.fam;
  a.Tr = s.Tr;
  a.Z = s.Z;
  a.XZ_part = s.XZ_part;
  a.ZTr_part = s.ZTr_part;
  a.key = s.key;
  a.iter = iter;
  a.iter_dev = s.capturing ? s.d_iter : nullptr;
  a.noise_zero = s.noise_mode;
  a.zprev_is_e = use_raw_y;  // only the init draw reads hM$Y (R/computeInitialParameters.R:254)
  a.mask_na = s.phylo ? 0 : 1;
  a.kt = s.kt_on ? s.d_kt + (size_t)KT_Z * 2 * KT_SLOTS : nullptr;
  dim3 grid(s.ntile_j, nchunk);  // species blocks fastest (z_kernel.h)
  size_t smem = z_smem_bytes(s.K, s.nt);
  // HMSC_XZ_FOLD: XZ left as chunk partials, summed by the fused Gamma2 + BetaLambda launch
  // where it reads them (xz_src: the BetaLambda bodies' partial loads, Gamma2's species-block
  // partials of G2SB species), so no reduction launch sits between this launch and that one,
  // and the record pack rides along as this launch's last grid row (with NA the ZTr reduction
  // runs anyway, and a sharded chain all-reduces XZ sums).  Off by default: at four rounds of
  // z workgroups (capi.cpp) the reduction launch measured 6,677-6,713 sweeps/s against the
  // fold's 6,601-6,688 (its ~15 MB of partial loads land on the BetaLambda prologue), and at
  // three rounds the fold led by ~1 % (profiles/r05_fold_ab2.txt)
  const bool fold = draw && !s.has_na && !s.sharded && !s.phylo && gamma2_bl_fusion_ok(s) &&
                    getenv_flag("HMSC_XZ_FOLD");
  a.pack_row = 0;
  // The record pack is z's last grid row without the fold as well, so the slab launch after z
  // sums XZ only: its ntile_j pack workgroups dispatch last and overlap z's final round
  // (1000-step config 4: 6,852 sweeps/s against 6,761 with the pack in the slab launch,
  // three same-box rounds, profiles/r06_packrow_ab.txt; HMSC_Z_PACK_ROW=0 restores the latter)
  static const bool pack_row_env = []() {
    const char* v = getenv("HMSC_Z_PACK_ROW");
    return !(v && v[0] == '0');
  }();
  static const bool pack_first = getenv_flag("HMSC_Z_PACK_FIRST");
  if ((fold || (pack_row_env && draw && !s.sharded)) && s.pack_req && s.side_fused && s.capturing) {
    a.pack_row = pack_first ? 2 : 1;
    a.pack = record_pack_args(s, 1);
    grid.y += 1;
    s.pack_req = false;
    s.pack_done = true;
  }
  if (draw && s.g_pending) {  // G's Eta rows reduced on an extra first grid row
    a.gred_y0 = 1;
    a.gred_ntile = s.g_ntile;
    a.gred_nf = s.g_nf;
    a.gred_Kmax = s.Kmax;
    a.gred_groups = (s.K * s.g_nf + 63) / 64;
    a.gred_part = s.G_part;
    a.gred_XX = s.XX;
    a.gred_G = s.G;
    grid.y += 1;
    smem = std::max(smem, (size_t)256 * sizeof(double));
    s.g_pending = false;
  }
  {
    ProfScope ps(s, PROF_Z);
    if (draw && s.any_poisson) {
      if (s.has_na)
        z_dispatch<true, true, true>(s, grid, smem, a);
      else
        z_dispatch<true, false, true>(s, grid, smem, a);
    } else if (draw) {
      if (s.has_na)
        z_dispatch<true, true>(s, grid, smem, a);
      else
        z_dispatch<true, false>(s, grid, smem, a);
    } else {
      if (s.has_na)
        z_dispatch<false, true>(s, grid, smem, a);
      else
        z_dispatch<false, false>(s, grid, smem, a);
    }
    HIP_OK(hipGetLastError());
  }
  if (fold) {
    s.xz_parts = nchunk;
    return;
  }
  s.xz_parts = 0;
  // XZ and ZTr from their partials, one launch
  const int64_t nXZ = (int64_t)s.K * s.nsl, nZT = s.has_na ? (int64_t)s.ny * s.nt : 0;
  const SideGate gate = draw ? side_gate_next(s, iter) : SideGate{};
  // a sharded sweep: all-reduce A's species sums ride in this launch (sweep_sharded)
  State* g2s = (draw && s.g2s_slab_req && !s.has_na && (s.mask & HMSC_UP_GAMMA2)) ? &s : nullptr;
  if (draw && s.pack_req && (s.side_fused || sharded_pack_split(s)) && s.capturing) {
    launch_slab_sum2_pack(s, s.XZ_part, s.XZ, nXZ, nchunk, s.ZTr_part, s.ZTr, nZT, s.ntile_j, gate, g2s);
    s.pack_req = false;
    s.pack_done = true;
  } else {
    launch_slab_sum2(s.XZ_part, s.XZ, nXZ, nchunk, s.ZTr_part, s.ZTr, nZT, s.ntile_j, s.stream, gate, g2s);
  }
  s.g2s_slab = g2s != nullptr;
}

// the z kernel's tables in one device buffer: the log table, then z_draw_tables
int z_log_table_doubles() { return ZLOG_W * ZLOG_N + ZT_DOUBLES; }
void z_log_table_fill(double* t) {
  z_log_table(t);
  z_draw_tables(t + ZLOG_W * ZLOG_N);
}

void launch_update_z(State& s, uint32_t iter, bool use_raw_y) {
  run_z_fused(s, true, iter, use_raw_y);
  s.zt_valid = true;
}

void launch_zt_refresh(State& s) {
  run_z_fused(s, false, 0, false);
  s.zt_valid = true;
}

}  // namespace hmsc
