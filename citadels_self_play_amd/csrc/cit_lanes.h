// Internal launcher shared by cit_hip.hip and cit_lanes.hip (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CIT_LANES_MAX_G 64
int cit_rollout_lanes(uint32_t* games, uint32_t* mt, uint32_t* mt_idx, uint64_t* seer, int B, int max_steps, int G,
                      int32_t* steps, int32_t* winner, hipStream_t stream);
