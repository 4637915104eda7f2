// oracle/ref_instr.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Forced-include (-include) for a second, instrumented compile of the reference's own
// /root/reference/grid.cpp into oracle/_ref/obj/grid_instr.o (oracle/Makefile).  Nothing of
// the reference is restated or replaced: its headers are included first (their include
// guards then make grid.cpp's own #includes no-ops), and two function-like macros wrap the
// calls grid.cpp makes so the reference's OWN walk reports what it did:
//
//   GridIdx(x, y, z)          grid.h:41-42, called once per DDA iteration of Grid::Intersect
//                             (grid.cpp:243) -> rt_ref_cell(): counts the iteration and
//                             remembers the cell index (the accepted cell on a hit, the last
//                             cell walked on a miss)
//   IntersectRayTri(...)      triangle.h:15-107, called per list entry (grid.cpp:248-256)
//                             -> counts the ray/triangle test
//
// A macro is not re-expanded inside its own replacement, so the wrapped call is the
// reference's unchanged member / inline function.  The counters are per-thread; refdriver's
// "samples" command resets them before every Grid::Intersect.  The floating-point work is
// untouched, and gen_golden.py checks that this build's hit/tri/t/u/v/colour columns equal
// the uninstrumented refdriver's bit for bit.
#ifndef RT_REF_INSTR_H
#define RT_REF_INSTR_H

#include "types.h"
#include "lin_alg.h"
#include "mesh.h"
#include "grid.h"
#include "triangle.h"

struct RtRefWalk
{
    uint32 cell;    // last GridIdx evaluated by the walk, 0xFFFFFFFF before the first
    uint32 steps;   // GridIdx evaluations = DDA iterations
    uint32 tests;   // IntersectRayTri calls
};
extern thread_local RtRefWalk g_rt_ref_walk;

inline uint rt_ref_cell(uint idx)
{
    g_rt_ref_walk.cell = idx;
    g_rt_ref_walk.steps++;
    return idx;
}

#ifndef RT_REF_INSTR_NO_HOOKS     // refdriver itself only reads the counters
#define GridIdx(x, y, z) rt_ref_cell(GridIdx(x, y, z))
#define IntersectRayTri(...) (g_rt_ref_walk.tests++, IntersectRayTri(__VA_ARGS__))
#endif

#endif // RT_REF_INSTR_H
