// X11 CPU reference chain (csrc/cpu/x11_cpu.cpp); the gfx950 launchers are in
// otedama/x11_launch.h.
#pragma once
#include <cstddef>
#include <cstdint>

#include "otedama/job.h"

namespace otedama {
namespace x11 {
// X11(msg) -> 32 bytes; `trace` (11 * 64 bytes or null) receives every stage digest.
void x11(const uint8_t* msg, size_t len, uint8_t out[32], uint8_t* trace);
// Stage i (0 = BLAKE-512 ... 10 = ECHO-512) of the chain on an arbitrary message.
void stage(int i, const uint8_t* msg, size_t len, uint8_t out[64]);
// The bitsliced Luffa SubCrumb used by the chain equals the S-box table (all inputs, every bit lane).
bool luffa_sbox_selfcheck();
}  // namespace x11

constexpr int kX11StageCount = 11;
}  // namespace otedama
