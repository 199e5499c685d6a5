// MFMA helpers shared by the fused filtered-lrelu kernels (flrelu_mfma.hip: forward; flrelu_bwd_mfma.hip: backward):
// f16 / bf16 fragment types, transposed LDS reads, LDS-DMA from inline asm, packing.
#pragma once
#include "flrelu.h"

namespace ic2 {

typedef _Float16 fm_h2 __attribute__((ext_vector_type(2)));
typedef _Float16 fm_h4 __attribute__((ext_vector_type(4)));
typedef _Float16 fm_h8 __attribute__((ext_vector_type(8)));
typedef short fm_s4 __attribute__((ext_vector_type(4)));
typedef float fm_f4 __attribute__((ext_vector_type(4)));
typedef float fm_f2 __attribute__((ext_vector_type(2)));
typedef uint32_t v2u32_t __attribute__((ext_vector_type(2)));

constexpr int FM_TAPS = 276;
// the wide / strip kernels' table also holds the clamp-split horizontal taps: guh at [328, 352), gdgl at [428, 440)
// (zero guards around each: the tap reads reach 15 below and 63 above gu's base, 30 below and 47 above gdg's)
constexpr int FM_TAPS_CL = 476;
constexpr uint32_t FM_OOB = 0x7ffffff0u;  // buffer num_records = the zero-answer offset (per-sample image < 2 GiB)


__device__ __forceinline__ fm_s4 fm_tr_read(const uint32_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) fm_s4*)p);
}

// LDS-DMA of 16 B per lane (buffer_load_dwordx4 ... lds: lane l's bytes land at lds_dst + 16 l) issued from inline
// asm: the compiler then does not know an LDS write is in flight and inserts no vmcnt(0) in front of the next LDS
// read of an unrelated buffer (which it does for the builtin, turning a prefetch into a synchronous load).  The
// caller waits for it with an explicit s_waitcnt vmcnt before a barrier.
// The statement opens with the wait states the hardware needs before the DMA reads its SGPR operands, which the
// compiler pads for a builtin but cannot see inside asm: 5 after a VALU write of a descriptor SGPR (v_readlane /
// v_readfirstlane: the compiler restores spilled descriptors with v_readlane right before the statement) and 1 after
// the SALU write of M0.  Without them the DMA can take a stale descriptor -- zeros (out of range) or a fault -- the
// cause of the round-3 oscale-row failures (DESIGN.md "LDS-DMA wait states").
__device__ __forceinline__ void fm_dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, const uint32_t* lds_dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint32_t*)lds_dst);
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "{m0}"(m0) : "memory");
}

// f32 -> f16 pairs (v_cvt_pk_f16_f32, round to nearest even)
__device__ __forceinline__ uint32_t fm_h2u(float a, float b) {
  return __builtin_bit_cast(uint32_t, fm_h2{(_Float16)a, (_Float16)b});
}
__device__ __forceinline__ uint2 fm_pack4(float a, float b, float c, float d) {
  return make_uint2(fm_h2u(a, b), fm_h2u(c, d));
}
__device__ __forceinline__ fm_h4 fm_h4_of(uint2 u) { return __builtin_bit_cast(fm_h4, u); }
__device__ __forceinline__ fm_h8 fm_h8_of(uint2 lo, uint2 hi) {
  return __builtin_bit_cast(fm_h8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

__device__ __forceinline__ int fm_xcd_remap(int b, int nblocks) {
  const int xcd = b & 7, loc = b >> 3;
  const int q8 = nblocks >> 3, r8 = nblocks & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
}

// Strip segmentation of the persistent strip kernels (forward flrelu_mfma3, backward flrelu_bwd_mfma): the grid of
// `resident` workgroups takes the nstrips * nseg items round-robin, so a launch lasts ceil(items / resident) rounds
// of one item.  Base rule (round 3): whole strips when there are >= 2 per resident workgroup, else the fewest
// segments that give 2.  `tune`: on strips of <= 40 tiles, the segmentation that minimises rounds x (segment tiles +
// a per-item start cost of about one tile: the ring prologue and the halo rows above the segment) -- whole strips
// on 2.1-2.5 items per workgroup idle much of the chip in the last round (SG3-T-1024 L5 / L6 / L8 / L9 -9 / -5 / -11
// / -15 %, profiles/r4zp_flr_segments_ab.txt); the 1044^2 layers' 66-tile strips measured level to 11 % slower cut.
inline int fm_strip_segments(int64_t nstrips, int tiles_y, int resident, bool tune) {
  int64_t nseg = (2 * (int64_t)resident + nstrips - 1) / nstrips;
  nseg = nseg < 1 ? 1 : (nseg > tiles_y ? tiles_y : nseg);
  if (tune && tiles_y <= 40) {
    int64_t best = -1, pick = nseg;
    for (int64_t sg = nseg; sg <= tiles_y && sg <= nseg + 16; ++sg) {
      const int64_t len = (tiles_y + sg - 1) / sg, segs = (tiles_y + len - 1) / len;
      const int64_t cost = (nstrips * segs + resident - 1) / resident * (len + 1);
      if (best < 0 || cost < best) best = cost, pick = segs;
    }
    nseg = pick;
  }
  return (int)nseg;
}

}  // namespace ic2
