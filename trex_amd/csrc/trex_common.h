// Shared constants and error plumbing for libtrexhip.so (host side).
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/trex_hip.h"

namespace trex {

constexpr int32_t kPlanMagic = 0x54524558;  // 'TREX'

// forward-step child descriptor: index bits 0-15, slot 16-23, kind 24-25
constexpr int32_t kStepAccumulate = 1 << 26;  // adjoint: add into the slot
// forward-step flags (word 3)
constexpr int32_t kStepRoot = 1;
constexpr int32_t kStepUnreached = 2;

// backtrack entry kinds (bits 16-19 of word 0)
constexpr int kBtRoot = 0;
constexpr int kBtReal = 1;
constexpr int kBtSentinel = 2;
constexpr int kBtUnreached = 3;

int set_error(int code, const char* fmt, ...);

}  // namespace trex
