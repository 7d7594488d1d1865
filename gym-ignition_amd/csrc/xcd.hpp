// xcd.hpp -- XCD-aware workgroup -> data block mapping for gfx950.
//
// The dispatcher hands workgroups to the 8 XCDs round-robin (workgroup b runs
// on XCD b % 8) and every XCD has its own L2.  Kernels whose neighbouring
// workgroups share cache lines (one world per wave or per 16-lane row, state
// laid out [dof][world]: a 128-B line holds 32 worlds) would otherwise make
// every XCD fetch and partially write every line.  xcd_block() renumbers the
// workgroups so that each XCD gets one contiguous range of blocks (a
// bijection on [0, gridDim.x) for any grid size).
#pragma once

#include <hip/hip_runtime.h>

namespace mw {
namespace dev {

__device__ __forceinline__ int xcd_block() {
    const int nb = static_cast<int>(gridDim.x), bx = static_cast<int>(blockIdx.x);
    const int q = nb >> 3, r = nb & 7, x = bx & 7;
    return x * q + (x < r ? x : r) + (bx >> 3);
}

}  // namespace dev
}  // namespace mw
