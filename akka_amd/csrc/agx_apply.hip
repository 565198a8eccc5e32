// agx_apply.hip — k_bucket_apply instantiations of one variant group (agx_variants.h).
// Built once per group with -DAGX_VGROUP=g; the unit with AGX_VGROUP_DISPATCH also holds the
// dispatcher agx_launch_apply() that routes a variant id to its group.
#include <hip/hip_runtime.h>

#include "agx_variants.h"

#ifndef AGX_VGROUP
#error "build agx_apply.hip with -DAGX_VGROUP=<group>"
#endif

#define AGX_CAT2(a, b) a##b
#define AGX_CAT(a, b) AGX_CAT2(a, b)
#define AGX_GROUP_FN AGX_CAT(agx_launch_apply_g, AGX_VGROUP)

namespace agx {

hipError_t agx_launch_apply_g0(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g1(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g2(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g3(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g4(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g5(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g6(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_apply_g7(uint32_t, uint32_t, bool, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g0(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g1(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g2(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g3(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g4(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g5(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g6(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_tiny_g7(uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g0(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g1(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g2(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g3(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g4(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g5(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g6(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_dense_g7(uint32_t, uint32_t, dim3, hipStream_t, const BucketArgs&);
hipError_t agx_launch_ring_g0(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g1(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g2(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g3(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g4(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g5(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g6(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_launch_ring_g7(uint32_t, bool, dim3, hipStream_t, const BucketArgs&, const RingArgs&);
hipError_t agx_dense_persist_occupancy_g0(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g1(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g2(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g3(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g4(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g5(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g6(uint32_t, int*);
hipError_t agx_dense_persist_occupancy_g7(uint32_t, int*);
static_assert(kVGroups == 8, "one declaration per group");

namespace {

template <uint32_t V>
hipError_t launch_v(uint32_t mode, bool skew, dim3 g, hipStream_t s, const BucketArgs& ba) {
  constexpr bool W = kVariants[V].wide;
  constexpr uint32_t M = kVariants[V].km;
  const dim3 blk(kBThreads);
  switch (mode * 2 + (skew ? 1u : 0u)) {
    case M_FUSED * 2: hipLaunchKernelGGL((k_bucket_apply<W, M, true, false, false>), g, blk, 0, s, ba); break;
    case M_FUSED * 2 + 1: hipLaunchKernelGGL((k_bucket_apply<W, M, true, true, false>), g, blk, 0, s, ba); break;
    case M_OWNER * 2: hipLaunchKernelGGL((k_bucket_apply<W, M, false, false, true>), g, blk, 0, s, ba); break;
    case M_OWNER * 2 + 1: hipLaunchKernelGGL((k_bucket_apply<W, M, false, true, true>), g, blk, 0, s, ba); break;
    case M_BYPASS * 2: hipLaunchKernelGGL((k_bucket_apply<W, M, false, false, false>), g, blk, 0, s, ba); break;
    case M_BYPASS * 2 + 1: hipLaunchKernelGGL((k_bucket_apply<W, M, false, true, false>), g, blk, 0, s, ba); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// the variants of this group, V in [0, V_N)
template <uint32_t V>
hipError_t group_dispatch(uint32_t vid, uint32_t mode, bool skew, dim3 g, hipStream_t s, const BucketArgs& ba) {
  if constexpr (V >= V_N) {
    return hipErrorInvalidValue;
  } else {
    if constexpr (kVariantGroup[V] == AGX_VGROUP)
      if (vid == V) return launch_v<V>(mode, skew, g, s, ba);
    return group_dispatch<V + 1>(vid, mode, skew, g, s, ba);
  }
}

// k_tiny_apply of the plain / compiled variants of this group
template <uint32_t V>
hipError_t tiny_dispatch(uint32_t vid, dim3 g, hipStream_t s, const BucketArgs& ba) {
  if constexpr (V >= V_N) {
    return hipErrorInvalidValue;
  } else {
    if constexpr (kVariantGroup[V] == AGX_VGROUP && !kVariants[V].wide)
      if (vid == V) {
        hipLaunchKernelGGL((k_tiny_apply<kVariants[V].km>), g, dim3(kTinyThreads), 0, s, ba);
        return hipGetLastError();
      }
    return tiny_dispatch<V + 1>(vid, g, s, ba);
  }
}

// k_ring_apply (tiny: k_ring_tiny) of the plain / compiled variants of this group
template <uint32_t V>
hipError_t dense_dispatch(uint32_t vid, uint32_t mode, dim3 g, hipStream_t s, const BucketArgs& ba) {
  if constexpr (V >= V_N) {
    return hipErrorInvalidValue;
  } else {
    if constexpr (kVariantGroup[V] == AGX_VGROUP && !kVariants[V].wide)
      if (vid == V) {
        if (mode == M_FUSED)
          hipLaunchKernelGGL((k_dense_fused<kVariants[V].km, false>), g, dim3(kDenseThreads), 0, s, ba);
        else if (mode == M_PERSIST)
          hipLaunchKernelGGL((k_dense_fused<kVariants[V].km, false, true>), g, dim3(kDenseThreads), 0, s, ba);
        else if (mode == M_OWNER)
          hipLaunchKernelGGL((k_dense_fused<kVariants[V].km, true>), g, dim3(kDenseThreads), 0, s, ba);
        else
          hipLaunchKernelGGL((k_dense_apply<kVariants[V].km>), g, dim3(kDenseThreads), 0, s, ba);
        return hipGetLastError();
      }
    return dense_dispatch<V + 1>(vid, mode, g, s, ba);
  }
}

template <uint32_t V>
hipError_t persist_occ(uint32_t vid, int* n) {
  if constexpr (V >= V_N) {
    return hipErrorInvalidValue;
  } else {
    if constexpr (kVariantGroup[V] == AGX_VGROUP && !kVariants[V].wide)
      if (vid == V)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(n, k_dense_fused<kVariants[V].km, false, true>,
                                                            kDenseThreads, 0);
    return persist_occ<V + 1>(vid, n);
  }
}

template <uint32_t V>
hipError_t ring_dispatch(uint32_t vid, bool tiny, dim3 g, hipStream_t s, const BucketArgs& ba, const RingArgs& ra) {
  if constexpr (V >= V_N) {
    return hipErrorInvalidValue;
  } else {
    if constexpr (kVariantGroup[V] == AGX_VGROUP && !kVariants[V].wide)
      if (vid == V) {
        if (tiny)
          hipLaunchKernelGGL((k_ring_tiny<kVariants[V].km>), g, dim3(kTinyThreads), 0, s, ba, ra);
        else
          hipLaunchKernelGGL((k_ring_apply<kVariants[V].km>), g, dim3(kBThreads), 0, s, ba, ra);
        return hipGetLastError();
      }
    return ring_dispatch<V + 1>(vid, tiny, g, s, ba, ra);
  }
}

}  // namespace

hipError_t AGX_CAT(agx_launch_ring_g, AGX_VGROUP)(uint32_t vid, bool tiny, dim3 g, hipStream_t s, const BucketArgs& ba,
                                                  const RingArgs& ra) {
  return ring_dispatch<0>(vid, tiny, g, s, ba, ra);
}

hipError_t AGX_CAT(agx_dense_persist_occupancy_g, AGX_VGROUP)(uint32_t vid, int* n) { return persist_occ<0>(vid, n); }

hipError_t AGX_CAT(agx_launch_tiny_g, AGX_VGROUP)(uint32_t vid, dim3 g, hipStream_t s, const BucketArgs& ba) {
  return tiny_dispatch<0>(vid, g, s, ba);
}

hipError_t AGX_CAT(agx_launch_dense_g, AGX_VGROUP)(uint32_t vid, uint32_t mode, dim3 g, hipStream_t s,
                                                   const BucketArgs& ba) {
  return dense_dispatch<0>(vid, mode, g, s, ba);
}

hipError_t AGX_GROUP_FN(uint32_t vid, uint32_t mode, bool skew, dim3 g, hipStream_t s, const BucketArgs& ba) {
  return group_dispatch<0>(vid, mode, skew, g, s, ba);
}

#if AGX_VGROUP == 0
hipError_t agx_launch_apply(uint32_t vid, uint32_t mode, bool skew, dim3 g, hipStream_t s, const BucketArgs& ba) {
  if (vid >= V_N) return hipErrorInvalidValue;
  switch (kVariantGroup[vid]) {
    case 0: return agx_launch_apply_g0(vid, mode, skew, g, s, ba);
    case 1: return agx_launch_apply_g1(vid, mode, skew, g, s, ba);
    case 2: return agx_launch_apply_g2(vid, mode, skew, g, s, ba);
    case 3: return agx_launch_apply_g3(vid, mode, skew, g, s, ba);
    case 4: return agx_launch_apply_g4(vid, mode, skew, g, s, ba);
    case 5: return agx_launch_apply_g5(vid, mode, skew, g, s, ba);
    case 6: return agx_launch_apply_g6(vid, mode, skew, g, s, ba);
    default: return agx_launch_apply_g7(vid, mode, skew, g, s, ba);
  }
}
hipError_t agx_launch_ring(uint32_t vid, bool tiny, dim3 g, hipStream_t s, const BucketArgs& ba, const RingArgs& ra) {
  if (vid >= V_N || kVariants[vid].wide) return hipErrorInvalidValue;
  switch (kVariantGroup[vid]) {
    case 0: return agx_launch_ring_g0(vid, tiny, g, s, ba, ra);
    case 1: return agx_launch_ring_g1(vid, tiny, g, s, ba, ra);
    case 2: return agx_launch_ring_g2(vid, tiny, g, s, ba, ra);
    case 3: return agx_launch_ring_g3(vid, tiny, g, s, ba, ra);
    case 4: return agx_launch_ring_g4(vid, tiny, g, s, ba, ra);
    case 5: return agx_launch_ring_g5(vid, tiny, g, s, ba, ra);
    case 6: return agx_launch_ring_g6(vid, tiny, g, s, ba, ra);
    default: return agx_launch_ring_g7(vid, tiny, g, s, ba, ra);
  }
}

hipError_t agx_launch_dense(uint32_t vid, uint32_t mode, dim3 g, hipStream_t s, const BucketArgs& ba) {
  if (vid >= V_N || kVariants[vid].wide) return hipErrorInvalidValue;
  switch (kVariantGroup[vid]) {
    case 0: return agx_launch_dense_g0(vid, mode, g, s, ba);
    case 1: return agx_launch_dense_g1(vid, mode, g, s, ba);
    case 2: return agx_launch_dense_g2(vid, mode, g, s, ba);
    case 3: return agx_launch_dense_g3(vid, mode, g, s, ba);
    case 4: return agx_launch_dense_g4(vid, mode, g, s, ba);
    case 5: return agx_launch_dense_g5(vid, mode, g, s, ba);
    case 6: return agx_launch_dense_g6(vid, mode, g, s, ba);
    default: return agx_launch_dense_g7(vid, mode, g, s, ba);
  }
}

hipError_t agx_dense_persist_occupancy(uint32_t vid, int* n) {
  *n = 0;
  if (vid >= V_N || kVariants[vid].wide) return hipErrorInvalidValue;
  switch (kVariantGroup[vid]) {
    case 0: return agx_dense_persist_occupancy_g0(vid, n);
    case 1: return agx_dense_persist_occupancy_g1(vid, n);
    case 2: return agx_dense_persist_occupancy_g2(vid, n);
    case 3: return agx_dense_persist_occupancy_g3(vid, n);
    case 4: return agx_dense_persist_occupancy_g4(vid, n);
    case 5: return agx_dense_persist_occupancy_g5(vid, n);
    case 6: return agx_dense_persist_occupancy_g6(vid, n);
    default: return agx_dense_persist_occupancy_g7(vid, n);
  }
}

hipError_t agx_launch_tiny(uint32_t vid, dim3 g, hipStream_t s, const BucketArgs& ba) {
  if (vid >= V_N || kVariants[vid].wide) return hipErrorInvalidValue;
  switch (kVariantGroup[vid]) {
    case 0: return agx_launch_tiny_g0(vid, g, s, ba);
    case 1: return agx_launch_tiny_g1(vid, g, s, ba);
    case 2: return agx_launch_tiny_g2(vid, g, s, ba);
    case 3: return agx_launch_tiny_g3(vid, g, s, ba);
    case 4: return agx_launch_tiny_g4(vid, g, s, ba);
    case 5: return agx_launch_tiny_g5(vid, g, s, ba);
    case 6: return agx_launch_tiny_g6(vid, g, s, ba);
    default: return agx_launch_tiny_g7(vid, g, s, ba);
  }
}
#endif

}  // namespace agx
