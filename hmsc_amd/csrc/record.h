// The record pack of a sweep: pieces of the device state copied into a ring slot (capi.cpp
// record_after_sweep).  Shared by pack_kernel / slab_pack_kernel (kernels.hip) and the z
// launch's pack row (z_kernel.h).
#pragma once
#include <cstdint>

#include "../../include/hmsc_amd.h"

namespace hmsc {

struct PackPiece {
  const double* src;
  int64_t n;
  int64_t dst;
};
constexpr int MAX_PIECES = 8 + 2 * HMSC_MAX_LEVELS;
struct PackArgs {
  PackPiece p[MAX_PIECES];
  int npieces;
  double* slot;
  // graph replays: the slot follows from the device sweep counter and the run descriptor
  // {iter0, transient, thin, samples}; sweeps that are not recorded return at once
  const uint32_t* iter_dev;
  const int32_t* desc;
  int64_t slot_stride;
  int ring_slots;
};

__device__ __forceinline__ void pack_body(const PackArgs& a, int bid, int nb) {
  double* slot = a.slot;
  if (a.iter_dev) {
    const int it = (int)(*a.iter_dev - (uint32_t)a.desc[0]);
    const int transient = a.desc[1], thin = a.desc[2], samples = a.desc[3];
    if (it <= transient || (it - transient) % thin != 0) return;
    const int k = (it - transient) / thin - 1;
    if (k >= samples) return;
    slot += (int64_t)(k % a.ring_slots) * a.slot_stride;
  }
  for (int k = 0; k < a.npieces; ++k) {
    const PackPiece pc = a.p[k];
    for (int64_t e = bid * (int64_t)blockDim.x + threadIdx.x; e < pc.n; e += (int64_t)nb * blockDim.x)
      slot[pc.dst + e] = pc.src[e];
  }
}

}  // namespace hmsc
