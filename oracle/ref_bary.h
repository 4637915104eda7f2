// oracle/ref_bary.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Forced-include (-include) for a third compile of the reference's own /root/reference/grid.cpp
// into oracle/_ref/obj/grid_bary.o (oracle/Makefile): the walk's ray/triangle test becomes the
// reference's second one.  grid.cpp calls IntersectRayTri(origin, dir, v0, v1, v2, cur_t, cur_u,
// cur_v) once per list entry (grid.cpp:248-256) with the triangle in scope as `tri`
// (grid.cpp:245); its commented-out alternative (grid.cpp:442-449) is the same call to
// IntersectRayTriBarycentric with `tri.n` inserted after the vertices.  The macro below makes
// exactly that substitution -- the reference's own IntersectRayTriBarycentric (triangle.h:210-226),
// nothing restated -- and keeps ref_instr.h's counters (the cell index and the test count).
#ifndef RT_REF_BARY_H
#define RT_REF_BARY_H

#define RT_REF_INSTR_NO_HOOKS
#include "ref_instr.h"
#undef RT_REF_INSTR_NO_HOOKS

#define GridIdx(x, y, z) rt_ref_cell(GridIdx(x, y, z))
#define IntersectRayTri(o, d, a, b, c, t, u, v) \
    (g_rt_ref_walk.tests++, IntersectRayTriBarycentric(o, d, a, b, c, tri.n, t, u, v))

#endif // RT_REF_BARY_H
