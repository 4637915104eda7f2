// rt_device.h -- device-side restatement of the reference's per-sample arithmetic for gfx950.
//
// Parity rules (SURVEY.md §7 hazards H1-H12), enforced by the build flags in csrc/Makefile
// (-ffp-contract=off, no fast-math, default IEEE f32 denormals, correctly rounded f32
// div/sqrt) and by keeping the reference's operation order in every expression below.
// Each function cites the reference line it restates; tests/test_gpu_parity.py checks it
// against the oracle and against the reference's own known-answer vectors.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {

constexpr float kFltMax = 3.402823466e+38f;   // std::numeric_limits<float>::max()
constexpr uint32_t kNoTri = 0xFFFFFFFFu;

// x86 cvttss2si semantics for the reference's (int) / (uchar) casts (grid.h:46,
// lin_alg.h:128-130): NaN and out-of-range give INT_MIN; AMDGPU's v_cvt_i32_f32 would
// saturate instead (hazard H7).
__device__ __forceinline__ int cvt_i32_x86(float x)
{
    return (x >= -2147483648.0f && x < 2147483648.0f) ? int(x) : int(0x80000000u);
}

// lin_alg.h:125-132 ToBGRA8 (alpha 0)
__device__ __forceinline__ uint32_t pack_bgra8(float r, float g, float b)
{
    const uint32_t rc = r > 1.0f ? 255u : uint32_t(cvt_i32_x86(r * 255.0f)) & 255u;
    const uint32_t gc = g > 1.0f ? 255u : uint32_t(cvt_i32_x86(g * 255.0f)) & 255u;
    const uint32_t bc = b > 1.0f ? 255u : uint32_t(cvt_i32_x86(b * 255.0f)) & 255u;
    return rc << 16 | gc << 8 | bc;
}

// renderer.cpp:125-131 gamma: glibc powf(x, 0.5f) is replaced by the correctly rounded
// sqrtf.  oracle/gamma_exhaustive.c proves pack_bgra8 of both is identical for EVERY
// float in [0, 1.0078] (and both saturate above); the float colour differs by <= 1 ulp
// on 678,030 inputs (hazard H6).
__device__ __forceinline__ float gamma_half(float x) { return __builtin_sqrtf(x); }

// One channel of pack_bgra8 (lin_alg.h:128-130)
__device__ __forceinline__ uint32_t pack_channel(float c)
{
    return c > 1.0f ? 255u : uint32_t(cvt_i32_x86(c * 255.0f)) & 255u;
}

// The hardware square root (v_sqrt_f32, within 1 ulp, no correction steps).  NOT used by the
// kernels: rt_debug_gamma_check finds 80 non-negative floats whose packed byte differs from the
// correctly rounded sqrtf's (measured on MI355X), and the 1080p x 4 frames of scenes 0, 4, 6, 7 and
// 9 change with it.  Kept only for that check.
__device__ __forceinline__ float gamma_fast(float x) { return __builtin_amdgcn_sqrtf(x); }

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz)
{
    float d = 0.0f;
    d += ax * bx;
    d += ay * by;
    d += az * bz;
    return d;
}

// 1.0f / x without the v_div_scale / v_div_fmas / v_div_fixup wrapper of the correctly rounded
// division (12 VALU -> 3): the v_rcp_f32 estimate refined by one FMA Newton step.  The
// result equals the correctly rounded 1.0f / x for EVERY float x with 2^-126 <= |x| < 2^126,
// checked exhaustively on gfx950 (rt_debug_rcp_check, tests/test_gpu_parity.py); callers use
// it only inside that range.  The two FMAs are explicit, not contraction (hazard H1 concerns
// a * b + c in the reference's expressions, which stay separately rounded).
constexpr float kRcpLo = 1e-8f;              // below it triangle.h:77 rejects det anyway
constexpr float kRcpHi = 8.5070591730234616e+37f;   // 2^126 (exclusive): exponents 253/254 and
                                                    // subnormal x mismatch (measured)
__device__ __forceinline__ float rcp_nr(float x)
{
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}

// 1.0f / x where rcp_nr is proven equal to the correctly rounded division (2^-126 <= |x| < kRcpHi,
// rt_debug_rcp_check over every float); lanes outside that range (zero, denormal, huge, inf, NaN
// -- rare) take the division behind a wave-uniform branch, so the common wave pays only the vote.
// Same bits as 1.0f / x for every x.
__device__ __forceinline__ float rcp_exact(float x)
{
    float r = rcp_nr(x);
    const float ax = __builtin_fabsf(x);
    const bool ok = ax >= 0x1p-126f && ax < kRcpHi;
    if (__builtin_amdgcn_ballot_w64(!ok) != 0ull)
        r = ok ? r : 1.0f / x;
    return r;
}


// triangle.h:15-107 IntersectRayTri, non-culling branch. e1 = v1 - v0 and e2 = v2 - v0 are
// precomputed on the host with the same single IEEE subtraction (triangle.h:41-42).
__device__ __forceinline__ bool ray_tri_mt(float ox, float oy, float oz, float dx, float dy, float dz,
                                           float v0x, float v0y, float v0z,
                                           float e1x, float e1y, float e1z,
                                           float e2x, float e2y, float e2z,
                                           float& t, float& u, float& v)
{
    const float px = dy * e2z - dz * e2y;
    const float py = dz * e2x - dx * e2z;
    const float pz = dx * e2y - dy * e2x;
    const float det = e1x * px + e1y * py + e1z * pz;
    if (det > -0.00000001f && det < 0.00000001f) return false;
    const float inv_det = 1.0f / det;
    const float tx = ox - v0x, ty = oy - v0y, tz = oz - v0z;
    u = (tx * px + ty * py + tz * pz) * inv_det;
    if (u < 0.0f || u > 1.0f) return false;
    const float qx = ty * e1z - tz * e1y;
    const float qy = tz * e1x - tx * e1z;
    const float qz = tx * e1y - ty * e1x;
    v = (dx * qx + dy * qy + dz * qz) * inv_det;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
    return t >= 0.0f;
}

// Branch-free form of ray_tri_mt for the traversal loop: every quantity is computed with the
// same operations in the same order, and the early-outs of triangle.h:77-101 become one
// predicate.  For an accepted hit t, u, v are bit-identical to ray_tri_mt's; rejected
// lanes merely carry garbage the caller ignores.  No divergent branches -> no exec-mask
// bookkeeping per test (SQ counters: SALU ~ VALU in the branchy loop).
__device__ __forceinline__ bool ray_tri_mt_pred(float ox, float oy, float oz, float dx, float dy, float dz,
                                                float v0x, float v0y, float v0z,
                                                float e1x, float e1y, float e1z,
                                                float e2x, float e2y, float e2z,
                                                float& t, float& u, float& v)
{
    const float px = dy * e2z - dz * e2y;
    const float py = dz * e2x - dx * e2z;
    const float pz = dx * e2y - dy * e2x;
    const float det = e1x * px + e1y * py + e1z * pz;
    const float inv_det = 1.0f / det;
    const float tx = ox - v0x, ty = oy - v0y, tz = oz - v0z;
    u = (tx * px + ty * py + tz * pz) * inv_det;
    const float qx = ty * e1z - tz * e1y;
    const float qy = tz * e1x - tx * e1z;
    const float qz = tx * e1y - ty * e1x;
    v = (dx * qx + dy * qy + dz * qz) * inv_det;
    t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
    const bool det_ok = !(det > -0.00000001f && det < 0.00000001f);
    const bool u_ok = !(u < 0.0f || u > 1.0f);
    const bool v_ok = !(v < 0.0f || u + v > 1.0f);
    return det_ok & u_ok & v_ok & (t >= 0.0f);
}

// ray_tri_mt_pred with a wave-uniform early out: when no active lane passes the det and u
// checks (triangle.h:77-87) the q/v/t half is skipped for the whole wave.  A scalar branch
// (s_cbranch on a ballot), not a divergent one; results identical to ray_tri_mt_pred.
__device__ __forceinline__ bool ray_tri_mt_gated(float ox, float oy, float oz, float dx, float dy, float dz,
                                                 float v0x, float v0y, float v0z,
                                                 float e1x, float e1y, float e1z,
                                                 float e2x, float e2y, float e2z,
                                                 float& t, float& u, float& v)
{
    const float px = dy * e2z - dz * e2y;
    const float py = dz * e2x - dx * e2z;
    const float pz = dx * e2y - dy * e2x;
    const float det = e1x * px + e1y * py + e1z * pz;
    const float inv_det = 1.0f / det;
    const float tx = ox - v0x, ty = oy - v0y, tz = oz - v0z;
    u = (tx * px + ty * py + tz * pz) * inv_det;
    const bool ok1 = !(det > -0.00000001f && det < 0.00000001f) & !(u < 0.0f || u > 1.0f);
    if (!__any(ok1)) return false;
    const float qx = ty * e1z - tz * e1y;
    const float qy = tz * e1x - tx * e1z;
    const float qz = tx * e1y - ty * e1x;
    v = (dx * qx + dy * qy + dz * qz) * inv_det;
    t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
    return ok1 & !(v < 0.0f || u + v > 1.0f) & (t >= 0.0f);
}

// Per-camera record of one CSR reference for rays that share one origin (every primary ray of
// a frame starts at the camera, camera.h:43).  tvec = o - v0 and qvec = tvec x e1
// (triangle.h:82, 90) do not depend on the direction, so k_origin_pre computes them once per
// camera origin with the same operations; only the direction-dependent half of
// triangle.h:15-107 remains per ray.  Record: {e1.xyz, e2.x} {e2.yz, tvec.xy} {tvec.z, qvec.xyz}.

// ---- the per-camera record test (AUTO's hot loop) ---------------------------------------
// With one camera origin per frame, tvec = origin - v0 (triangle.h:82), qvec = tvec x edge1
// (:90) and DOT(edge2, qvec) (:98) are per-reference constants: k_origin_pre computes them once
// per camera with the reference's exact operations (make_frec) into a 64-byte record laid out
// for packed f32 math: every pair below is one 64-bit register operand of a v_pk_mul_f32 /
// v_pk_add_f32, which perform two IEEE single-precision operations -- the same roundings as two
// v_mul_f32 / v_add_f32 -- so the reference's bits are kept while the instruction count drops.
//
//   r0 = (e1x, tx, e1y, ty)   r1 = (e1z, tz, e2y, e2z)   r2 = (e2x, e2y, qx, qy)   r3 = (qz, tq, 0, 0)
//
// The ray enters as two VGPR pairs a = (dx, dy) and c = (dy, dz).
typedef float f2v __attribute__((ext_vector_type(2)));

struct FRec { float4 r0, r1, r2, r3; };

// k_origin_pre's arithmetic for one reference (v0, e1, e2 as in the scene's reference record).
__device__ __forceinline__ FRec make_frec(float ox, float oy, float oz, float v0x, float v0y, float v0z,
                                          float e1x, float e1y, float e1z, float e2x, float e2y, float e2z)
{
    const float tx = ox - v0x, ty = oy - v0y, tz = oz - v0z;   // triangle.h:82 SUB(tvec, origin, vert0)
    const float qx = ty * e1z - tz * e1y;                      // triangle.h:90 CROSS(qvec, tvec, edge1)
    const float qy = tz * e1x - tx * e1z;
    const float qz = tx * e1y - ty * e1x;
    const float tq = e2x * qx + e2y * qy + e2z * qz;           // triangle.h:98 DOT(edge2, qvec)
    FRec f;
    f.r0 = make_float4(e1x, tx, e1y, ty);
    f.r1 = make_float4(e1z, tz, e2y, e2z);
    f.r2 = make_float4(e2x, e2y, qx, qy);
    f.r3 = make_float4(qz, tq, 0.0f, 0.0f);
    return f;
}

// First half (triangle.h:45-87): pvec = dir x edge2, det = edge1 . pvec, u = tvec . pvec * inv_det.
// Products and sums in the reference's order, two lanes of each pair at a time:
//   (pz, px) = (dx*e2y, dy*e2z) - (dy*e2x, dz*e2y),   py = dz*e2x - dx*e2z
//   (det, u') = ((e1x, tx)*px + (e1y, ty)*py) + (e1z, tz)*pz
// FAST_RCP: inv_det by rcp_nr, exact wherever the result is used: |det| < 1e-8 is rejected, and
// the launch selects FAST_RCP only for scenes whose |e1|_1 |e2|_1 bounds |det| far below 2^126.
template <bool FAST_RCP>
__device__ __forceinline__ bool mt_rec_first(f2v a, f2v c, f2v e1t_x, f2v e1t_y, f2v e1t_z, f2v e2yz, f2v e2xy,
                                             float& inv_det, float& u)
{
    const f2v zx = a * e2yz - c * e2xy;                        // (pz, px)
    const float py = c.y * e2xy.x - a.x * e2yz.y;
    const f2v m = (e1t_x * zx.y + e1t_y * py) + e1t_z * zx.x;  // (det, DOT(tvec, pvec))
    const float det = m.x;
    inv_det = FAST_RCP ? rcp_nr(det) : 1.0f / det;
    u = m.y * inv_det;
    return !(det > -0.00000001f && det < 0.00000001f) & !(u < 0.0f || u > 1.0f);
}

// Second half (triangle.h:90-101): v = DOT(dir, qvec) * inv_det, t = DOT(edge2, qvec) * inv_det
// with the record's constant DOT(edge2, qvec).
__device__ __forceinline__ bool mt_rec_second(f2v a, f2v c, f2v qxy, float qz, float tq, float inv_det, float u,
                                              float& v, float& t)
{
    const f2v dq = a * qxy;
    v = ((dq.x + dq.y) + c.y * qz) * inv_det;
    t = tq * inv_det;
    return !(v < 0.0f || u + v > 1.0f) & (t >= 0.0f);
}

// The whole record test, wave-gated (the v/t half only when some lane passed det and u);
// results identical to ray_tri_mt_gated on the hits.
template <bool FAST_RCP>
__device__ __forceinline__ bool ray_tri_frec_gated(f2v a, f2v c, const FRec& r, float& t, float& u, float& v)
{
    float inv_det;
    const bool ok1 = mt_rec_first<FAST_RCP>(a, c, f2v{r.r0.x, r.r0.y}, f2v{r.r0.z, r.r0.w}, f2v{r.r1.x, r.r1.y},
                                            f2v{r.r1.z, r.r1.w}, f2v{r.r2.x, r.r2.y}, inv_det, u);
    if (!__any(ok1)) return false;
    return ok1 & mt_rec_second(a, c, f2v{r.r2.z, r.r2.w}, r.r3.x, r.r3.y, inv_det, u, v, t);
}

// triangle.h:200-226 IntersectRayPlane + ComputeBarycentric (:133-156). Uses v0, the same
// e1 (= v1 - v0) and e2 (= v2 - v0, the reference's e0) and the face normal.
__device__ __forceinline__ bool ray_tri_bary(float ox, float oy, float oz, float dx, float dy, float dz,
                                             float v0x, float v0y, float v0z,
                                             float e1x, float e1y, float e1z,
                                             float e2x, float e2y, float e2z,
                                             float nx, float ny, float nz,
                                             float& t, float& u, float& v)
{
    const float denom = dot3(nx, ny, nz, dx, dy, dz);
    if (__builtin_fabsf(denom) < 0.00000001f) return false;
    const float dd = dot3(nx, ny, nz, v0x, v0y, v0z);
    t = (dd - dot3(nx, ny, nz, ox, oy, oz)) / denom;
    if (!(t >= 0.0f)) return false;                              // t >= 0.0 (double compare)
    const float qx = ox + dx * t, qy = oy + dy * t, qz = oz + dz * t;
    const float wx = qx - v0x, wy = qy - v0y, wz = qz - v0z;     // e2 = pos - v0
    const float d00 = dot3(e2x, e2y, e2z, e2x, e2y, e2z);       // e0 = v2 - v0
    const float d01 = dot3(e2x, e2y, e2z, e1x, e1y, e1z);
    const float d02 = dot3(e2x, e2y, e2z, wx, wy, wz);
    const float d11 = dot3(e1x, e1y, e1z, e1x, e1y, e1z);
    const float d12 = dot3(e1x, e1y, e1z, wx, wy, wz);
    const float inv_denom = 1.0f / (d00 * d11 - d01 * d01);
    u = (d00 * d12 - d01 * d02) * inv_denom;
    v = (d11 * d02 - d01 * d12) * inv_denom;
    return (u >= 0.0f) && (v >= 0.0f) && (u + v < 1.0f);
}

// Branch-free form of ray_tri_bary (same operations; accepted results bit-identical).
__device__ __forceinline__ bool ray_tri_bary_pred(float ox, float oy, float oz, float dx, float dy, float dz,
                                                  float v0x, float v0y, float v0z,
                                                  float e1x, float e1y, float e1z,
                                                  float e2x, float e2y, float e2z,
                                                  float nx, float ny, float nz,
                                                  float& t, float& u, float& v)
{
    const float denom = dot3(nx, ny, nz, dx, dy, dz);
    const float dd = dot3(nx, ny, nz, v0x, v0y, v0z);
    t = (dd - dot3(nx, ny, nz, ox, oy, oz)) / denom;
    const float qx = ox + dx * t, qy = oy + dy * t, qz = oz + dz * t;
    const float wx = qx - v0x, wy = qy - v0y, wz = qz - v0z;
    const float d00 = dot3(e2x, e2y, e2z, e2x, e2y, e2z);
    const float d01 = dot3(e2x, e2y, e2z, e1x, e1y, e1z);
    const float d02 = dot3(e2x, e2y, e2z, wx, wy, wz);
    const float d11 = dot3(e1x, e1y, e1z, e1x, e1y, e1z);
    const float d12 = dot3(e1x, e1y, e1z, wx, wy, wz);
    const float inv_denom = 1.0f / (d00 * d11 - d01 * d01);
    u = (d00 * d12 - d01 * d02) * inv_denom;
    v = (d11 * d02 - d01 * d12) * inv_denom;
    const bool plane_ok = !(__builtin_fabsf(denom) < 0.00000001f) & (t >= 0.0f);
    return plane_ok & (u >= 0.0f) & (v >= 0.0f) & (u + v < 1.0f);
}

// triangle.h:163-172 LineSegMinDistSq(a, b, p); ab = b - a and len_sq = Dot(ab, ab) come
// precomputed (same single IEEE operations), Clamp is lin_alg.h:205-212 (NaN passes through).
__device__ __forceinline__ float seg_dist_sq(float ax, float ay, float az, float abx, float aby, float abz,
                                             float len_sq, float px, float py, float pz)
{
    float t = dot3(px - ax, py - ay, pz - az, abx, aby, abz) / len_sq;
    t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
    const float qx = ax + t * abx, qy = ay + t * aby, qz = az + t * abz;
    const float dx = px - qx, dy = py - qy, dz = pz - qz;
    return dot3(dx, dy, dz, dx, dy, dz);
}

// Per-triangle record of the distance kernels (6 float4, built by rt_scene_create):
//   {v0.xyz, v1.x} {v1.yz, v2.xy} {v2.z, e0.xyz} {e1.xyz, e12.x} {e12.yz, dot00, dot01}
//   {dot11, inv_denom, len12, 0}
// with e0 = v2 - v0, e1 = v1 - v0, e12 = v2 - v1 and the position-independent terms of
// ComputeBarycentric (triangle.h:140-150): dot00 = Dot(e0,e0), dot01 = Dot(e0,e1),
// dot11 = Dot(e1,e1), inv_denom = 1 / (dot00*dot11 - dot01*dot01); len12 = Dot(e12,e12).
// LineSegMinDistSq(v0,v1) / (v0,v2) reuse e1 / e0 and dot11 / dot00: the same operations.
//
// triangle.h:174-198 DistancePointTri(pos, v0, v1, v2)
__device__ __forceinline__ float dist_point_tri(float px, float py, float pz, const float4& r0, const float4& r1,
                                                const float4& r2, const float4& r3, const float4& r4,
                                                const float4& r5)
{
    const float v0x = r0.x, v0y = r0.y, v0z = r0.z, v1x = r0.w, v1y = r1.x, v1z = r1.y;
    const float v2x = r1.z, v2y = r1.w, v2z = r2.x;
    // ComputeBarycentric (triangle.h:133-156) with e2 = pos - v0
    const float wx = px - v0x, wy = py - v0y, wz = pz - v0z;
    const float dot02 = dot3(r2.y, r2.z, r2.w, wx, wy, wz);
    const float dot12 = dot3(r3.x, r3.y, r3.z, wx, wy, wz);
    const float dot00 = r4.z, dot01 = r4.w, dot11 = r5.x, inv_denom = r5.y;
    const float u = (dot00 * dot12 - dot01 * dot02) * inv_denom;
    const float v = (dot11 * dot02 - dot01 * dot12) * inv_denom;
    if ((u >= 0.0f) && (v >= 0.0f) && (u + v < 1.0f))
    {
        // BarycentricInterpolate (triangle.h:158-161): v1*u + v2*v + v0*(1 - u - v)
        const float w = 1.0f - u - v;
        const float qx = v1x * u + v2x * v + v0x * w;
        const float qy = v1y * u + v2y * v + v0y * w;
        const float qz = v1z * u + v2z * v + v0z * w;
        const float dx = px - qx, dy = py - qy, dz = pz - qz;
        return __builtin_sqrtf(dot3(dx, dy, dz, dx, dy, dz));   // Distance, lin_alg.h:149-150
    }
    const float l01 = seg_dist_sq(v0x, v0y, v0z, r3.x, r3.y, r3.z, dot11, px, py, pz);
    const float l02 = seg_dist_sq(v0x, v0y, v0z, r2.y, r2.z, r2.w, dot00, px, py, pz);
    const float l12 = seg_dist_sq(v1x, v1y, v1z, r3.w, r4.x, r4.y, r5.z, px, py, pz);
    const float inner = (l12 < l02) ? l12 : l02;                // std::min(l02, l12)
    return __builtin_sqrtf((inner < l01) ? inner : l01);         // std::min(l01, inner)
}

// aabb.h:9-13
__device__ __forceinline__ bool point_in_aabb(float px, float py, float pz, const float* mn, const float* mx)
{
    return px >= mn[0] && py >= mn[1] && pz >= mn[2] && px <= mx[0] && py <= mx[1] && pz <= mx[2];
}

// aabb.h:34-83 (Williams et al.); IEEE inf/NaN from 1/+-0 select the slab order (H3, H9)
__device__ __forceinline__ bool ray_aabb(float ox, float oy, float oz, float dx, float dy, float dz,
                                         const float* mn, const float* mx, float& tmin, float& tmax)
{
    const float ix = rcp_exact(dx), iy = rcp_exact(dy), iz = rcp_exact(dz);   // = 1.0f / d
    const bool sx = ix < 0.0f, sy = iy < 0.0f, sz = iz < 0.0f;
    tmin = ((sx ? mx[0] : mn[0]) - ox) * ix;
    tmax = ((sx ? mn[0] : mx[0]) - ox) * ix;
    const float tymin = ((sy ? mx[1] : mn[1]) - oy) * iy;
    const float tymax = ((sy ? mn[1] : mx[1]) - oy) * iy;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((sz ? mx[2] : mn[2]) - oz) * iz;
    const float tzmax = ((sz ? mn[2] : mx[2]) - oz) * iz;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return true;
}

// lin_alg.h:138-156 Dot (accumulates from T() = 0) and Normalize (1/sqrt, then scale; the
// reciprocal by rcp_exact: same bits as 1.0f / sqrt)
__device__ __forceinline__ void normalize3(float& x, float& y, float& z)
{
    float d = 0.0f;
    d += x * x;
    d += y * y;
    d += z * z;
    const float len = rcp_exact(__builtin_sqrtf(d));
    x = x * len;
    y = y * len;
    z = z * len;
}

// camera.h:39-46 from the camera-space (x, y) of a sample (z = -1): Normalize (lin_alg.h:151-156:
// 1/sqrt then scale; the reciprocal by rcp_exact, same bits) and Transf3x3 (lin_alg.h:495-509,
// row-vector convention: m[r][c], r = input component).
__device__ __forceinline__ void dir_from_xy(const float* m, float x, float y, float& dx, float& dy, float& dz)
{
    float z = -1.0f;
    float d = 0.0f;
    d += x * x;
    d += y * y;
    d += z * z;
    const float len = rcp_exact(__builtin_sqrtf(d));
    x = x * len;
    y = y * len;
    z = z * len;
    dx = x * m[0] + y * m[3] + z * m[6];
    dy = x * m[1] + y * m[4] + z * m[7];
    dz = x * m[2] + y * m[5] + z * m[8];
}

// camera.h:20-21, 40-42: the camera-space x of pixel column px / y of row py at sample offset
// (sx, sy).  The kernels read both from per-frame tables built on the host with these same
// operations (rt_scene's ndc tables: x depends on (px, s) only, y on (py, s) only).
__host__ __device__ __forceinline__ float cam_x(uint32_t px, float sx, uint32_t W, float fov_xs)
{
    const float ndc_x = (float(px) + sx) / float(W) * 2.0f - 1.0f;
    return ndc_x * fov_xs;
}
__host__ __device__ __forceinline__ float cam_y(uint32_t py, float sy, uint32_t H, float fov_xs, float aspect)
{
    const float ndc_y = (float(py) + sy) / float(H) * 2.0f - 1.0f;
    return ndc_y * fov_xs / aspect;
}

// camera.h:8-47 GenerateRay, perspective branch. The per-frame constants fov_xs
// (= (float)tan(double), hazard H5), aspect and the origin are computed on the host.
__device__ __forceinline__ void gen_dir(const float* m, float fov_xs, float aspect, uint32_t px, uint32_t py,
                                        uint32_t W, uint32_t H, float sx, float sy,
                                        float& dx, float& dy, float& dz)
{
    dir_from_xy(m, cam_x(px, sx, W, fov_xs), cam_y(py, sy, H, fov_xs, aspect), dx, dy, dz);
}

// triangle.h:158-161 + lin_alg.h:151-156 + renderer.cpp:110-117
__device__ __forceinline__ void shade_hit(float u, float v, const float4& a, const float4& b, const float4& c,
                                          float& r, float& g, float& bl)
{
    // a = {n0.x, n0.y, n0.z, n1.x}, b = {n1.y, n1.z, n2.x, n2.y}, c = {n2.z, -, -, -}
    const float w = 1.0f - u - v;
    float x = a.w * u + b.z * v + a.x * w;
    float y = b.x * u + b.w * v + a.y * w;
    float z = b.y * u + c.x * v + a.z * w;
    normalize3(x, y, z);
    r = (x + 1.0f) * 0.5f;
    g = (y + 1.0f) * 0.5f;
    bl = (z + 1.0f) * 0.5f;
}

} // namespace rtd
