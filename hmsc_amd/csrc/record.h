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
  // kernel record copies (State::kcopy, graph replays): the slot is written through (device
  // scope) and the last workgroup of the pack raises flags[slot] = (run nonce desc[4] << 32 |
  // sample + 1) for the copy kernel (rec_copy_kernel) that moves the slot to the host ring
  uint64_t* flags;
  int* ticket;
};

__device__ __forceinline__ void pack_body(const PackArgs& a, int bid, int nb) {
  double* slot = a.slot;
  int ks = -1;
  if (a.iter_dev) {
    const int it = (int)(*a.iter_dev - (uint32_t)a.desc[0]);
    const int transient = a.desc[1], thin = a.desc[2], samples = a.desc[3];
    if (it <= transient || (it - transient) % thin != 0) return;
    const int k = (it - transient) / thin - 1;
    if (k >= samples) return;
    ks = k;
    slot += (int64_t)(k % a.ring_slots) * a.slot_stride;
  }
  const bool flag = a.flags && ks >= 0;
  for (int k = 0; k < a.npieces; ++k) {
    const PackPiece pc = a.p[k];
    for (int64_t e = bid * (int64_t)blockDim.x + threadIdx.x; e < pc.n; e += (int64_t)nb * blockDim.x) {
      if (flag)
        __hip_atomic_store((unsigned long long*)(slot + pc.dst + e), (unsigned long long)__double_as_longlong(pc.src[e]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        slot[pc.dst + e] = pc.src[e];
    }
  }
  if (flag) {  // every workgroup's write-through stores done, then a ticket; the last raises the flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(a.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
      __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.flags + ks % a.ring_slots, ((unsigned long long)(uint32_t)a.desc[4] << 32) | (uint32_t)(ks + 1),
                         __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace hmsc
