// agx_variants.h — the k_bucket_apply instantiations the engine launches, and where they live.
//
// Every (behaviour-mask variant, pipeline mode, fast/skew) combination is a separate kernel
// (k_bucket_apply<kWide, KM, kGather, kSkew, kOwner>, agx_kernels.h).  They are instantiated in
// agx_apply.hip, which the build compiles once per variant group (-DAGX_VGROUP=g), so the ~100
// kernels compile in parallel translation units instead of one; the host runtime
// (agx_engine.hip) only calls agx_launch_apply().
#pragma once
#include "agx_kernels.h"

namespace agx {

struct ApplyVariant {
  bool wide;    // CRDT state gossips (snapshot heap) possible
  uint32_t km;  // behaviour-kind mask the variant is specialised to
};

constexpr uint32_t kCrdtKM = kb(AGX_KIND_GCOUNTER) | kb(AGX_KIND_PNCOUNTER) | kb(AGX_KIND_ORSET);

// variant ids (the engine picks one from the registered kinds, agx_engine.hip launch_apply)
enum : uint32_t {
  V_GC_DELTA = 0, V_PN_DELTA, V_OR_DELTA, V_ALL_DELTA,
  V_GC, V_PN, V_OR, V_CRDT, V_ALL_WIDE,
  V_RING, V_FWD, V_FANOUT, V_COUNTER, V_COMPILED, V_ALL_COMPILED, V_ALL,
  V_N
};
constexpr ApplyVariant kVariants[V_N] = {
    {true, kb(AGX_KIND_GCOUNTER) | kDeltaKM}, {true, kb(AGX_KIND_PNCOUNTER) | kDeltaKM},
    {true, kb(AGX_KIND_ORSET) | kDeltaKM},    {true, KM_ALL | kDeltaKM},
    {true, kb(AGX_KIND_GCOUNTER)},            {true, kb(AGX_KIND_PNCOUNTER)},
    {true, kb(AGX_KIND_ORSET)},               {true, kCrdtKM},
    {true, KM_ALL},                           {false, kb(AGX_KIND_RING)},
    {false, kb(AGX_KIND_FORWARD_RR)},         {false, kb(AGX_KIND_FANOUT)},
    {false, kb(AGX_KIND_COUNTER)},            {false, kb(AGX_KIND_COMPILED)},
    {false, KM_ALL | kb(AGX_KIND_COMPILED)},  {false, KM_ALL},
};

// pipeline modes: fused single-rank gather (kGather), multi-rank owner grouping (kOwner),
// single-rank multi-pass with the backlog in place (neither)
enum : uint32_t { M_FUSED = 0, M_OWNER = 1, M_BYPASS = 2, M_PERSIST = 3 /* dense launch only: k_dense_fused<.., true> */ };

// variant groups = translation units (agx_apply.hip built with -DAGX_VGROUP=0..kVGroups-1);
// the heavy CRDT variants are spread so the units take similar time
constexpr uint32_t kVGroups = 8;
constexpr uint32_t kVariantGroup[V_N] = {0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 3, 4, 5, 6, 7};

// launch k_bucket_apply<variant vid, mode, skew> with `grid` x kBThreads threads on `s`
// (defined in agx_apply.hip; returns hipErrorInvalidValue for an unknown combination)
hipError_t agx_launch_apply(uint32_t vid, uint32_t mode, bool skew, dim3 grid, hipStream_t s, const BucketArgs& ba);
// launch k_tiny_apply<variant vid's kinds> (plain / compiled variants only: hipErrorInvalidValue otherwise)
hipError_t agx_launch_tiny(uint32_t vid, dim3 grid, hipStream_t s, const BucketArgs& ba);
// launch k_dense_apply<variant vid's kinds> (mode M_FUSED / M_OWNER: k_dense_fused) (plain / compiled variants only)
hipError_t agx_launch_dense(uint32_t vid, uint32_t mode, dim3 grid, hipStream_t s, const BucketArgs& ba);
// resident blocks per CU of the persistent fused dense launch of variant vid (0: not a dense variant)
hipError_t agx_dense_persist_occupancy(uint32_t vid, int* blocks_per_cu);
// launch k_ring_apply<variant vid's kinds> (tiny: k_ring_tiny, kTinyThreads) (plain / compiled variants only)
hipError_t agx_launch_ring(uint32_t vid, bool tiny, dim3 grid, hipStream_t s, const BucketArgs& ba, const RingArgs& ra);

}  // namespace agx
