// gfx950 X11 stage launchers (csrc/kernels/x11_stages_{a,b}.hip); HIP translation units only.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "otedama/hitsink.h"
#include "otedama/job.h"

namespace otedama {


// Stage i on the GPU over nonces base .. base + n - 1. H holds the 64-byte
// intermediate digests as 8 planes of u64 (word w of nonce k at H[w * stride + k]).
// Stage 0 reads the header from `p`; stage 10 with sink != null compares with the
// target and publishes nonces to *sink (otedama/hitsink.h) instead of writing H. Every
// stage honours the sink's abort word.
hipError_t x11_launch_stage(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                            const HitSink* sink, hipStream_t s);
hipError_t x11_launch_chain(const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                            const HitSink* sink, hipStream_t s);
}  // namespace otedama
