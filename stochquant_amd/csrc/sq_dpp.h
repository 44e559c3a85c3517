// sq_dpp.h -- wave-level helpers on DPP lane moves (no LDS round trips),
// shared by the QM1D kernels (sq_qm1d.hip, sq_qm1d_gs.hip) and the phi^4
// frame records (sq_phi4.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace sq {
namespace {

// Wave-wide max-scans by DPP (row_shr 1/2/4/8, row_bcast 15/31: the gfx9
// inclusive-scan sequence), no LDS round trips; 64-bit values move as two
// 32-bit DPP halves.  Out-of-range lanes read the identity (bound_ctrl off).
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_d(double v, double id) {
    const int lo = __builtin_amdgcn_update_dpp((int)__double2loint(id), (int)__double2loint(v), CTRL, RM, BM, false);
    const int hi = __builtin_amdgcn_update_dpp((int)__double2hiint(id), (int)__double2hiint(v), CTRL, RM, BM, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_i(int v, int id) {
    return __builtin_amdgcn_update_dpp(id, v, CTRL, RM, BM, false);
}
// v_max_f64 as is: fmax of a DPP-moved value (integer moves to the compiler)
// gets a quieting v_max_f64 x, x, x per operand first; the scanned values are
// results of arithmetic, never signalling NaNs, and a quiet NaN still yields
// the other operand
__device__ __forceinline__ double dpp_vmax_d(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// A lane with no source lane (or a row the mask leaves out) keeps the moved
// register's previous contents instead of a fresh -inf: that register only
// ever holds -inf or a value moved from a lower lane, which the inclusive
// maximum already covers, so the scan is unchanged and the two moves of the
// identity per stage go away.
__device__ __forceinline__ double dpp_incl_max(double v) {
    double t = -__builtin_inf();
    t = dpp_d<0x111, 0xf, 0xf>(v, t);
    v = dpp_vmax_d(v, t);
    t = dpp_d<0x112, 0xf, 0xf>(v, t);
    v = dpp_vmax_d(v, t);
    t = dpp_d<0x114, 0xf, 0xf>(v, t);
    v = dpp_vmax_d(v, t);
    t = dpp_d<0x118, 0xf, 0xf>(v, t);
    v = dpp_vmax_d(v, t);
    t = dpp_d<0x142, 0xa, 0xf>(v, t);
    v = dpp_vmax_d(v, t);
    t = dpp_d<0x143, 0xc, 0xf>(v, t);
    return dpp_vmax_d(v, t);
}
__device__ __forceinline__ double dpp_excl_max(double v) {  // max over lanes < this lane
    return dpp_d<0x138, 0xf, 0xf>(dpp_incl_max(v), -__builtin_inf());  // wave_shr:1
}
__device__ __forceinline__ double dpp_all_max(double v) {
    const double s = dpp_incl_max(v);
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(s), 63),
                            __builtin_amdgcn_readlane(__double2loint(s), 63));
}
__device__ __forceinline__ int dpp_all_max_i(int v) {
    const int id = (int)0x80000000;
    v = max(v, dpp_i<0x111, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x112, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x114, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x118, 0xf, 0xf>(v, id));
    v = max(v, dpp_i<0x142, 0xa, 0xf>(v, id));
    v = max(v, dpp_i<0x143, 0xc, 0xf>(v, id));
    return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int dpp_all_min_i(int v) { return -dpp_all_max_i(-v); }
template <int CTRL, int RM, int BM>
__device__ __forceinline__ unsigned long long dpp_max_step_u64(unsigned long long v) {
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)v, CTRL, RM, BM, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(v >> 32), CTRL, RM, BM, false);
    const unsigned long long w = ((unsigned long long)hi << 32) | lo;
    return w > v ? w : v;
}
__device__ __forceinline__ unsigned long long dpp_all_max_u64(unsigned long long v) {  // wave-uniform
    v = dpp_max_step_u64<0x111, 0xf, 0xf>(v);
    v = dpp_max_step_u64<0x112, 0xf, 0xf>(v);
    v = dpp_max_step_u64<0x114, 0xf, 0xf>(v);
    v = dpp_max_step_u64<0x118, 0xf, 0xf>(v);
    v = dpp_max_step_u64<0x142, 0xa, 0xf>(v);
    v = dpp_max_step_u64<0x143, 0xc, 0xf>(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ float dpp_f(float v, float id) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, id), __builtin_bit_cast(int, v),
                                                                 CTRL, RM, BM, false));
}
// v_max_f32 as is: fmaxf of a DPP-moved value (an integer move to the
// compiler) gets a quieting v_max_f32 x, x, x first; the moved values here are
// never signalling NaNs
__device__ __forceinline__ float dpp_vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float dpp_all_max_f(float v) {  // wave maximum (no NaN inputs), wave-uniform
    const float id = -__builtin_inff();
    v = dpp_vmax(v, dpp_f<0x111, 0xf, 0xf>(v, id));
    v = dpp_vmax(v, dpp_f<0x112, 0xf, 0xf>(v, id));
    v = dpp_vmax(v, dpp_f<0x114, 0xf, 0xf>(v, id));
    v = dpp_vmax(v, dpp_f<0x118, 0xf, 0xf>(v, id));
    v = dpp_vmax(v, dpp_f<0x142, 0xa, 0xf>(v, id));
    v = dpp_vmax(v, dpp_f<0x143, 0xc, 0xf>(v, id));
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// lane l <- lane l-1 (wave_shr:1) / lane l+1 (wave_shl:1); the lane shifted
// in from outside the wave keeps `id`
__device__ __forceinline__ double dpp_from_left(double v, double id) { return dpp_d<0x138, 0xf, 0xf>(v, id); }
__device__ __forceinline__ double dpp_from_right(double v, double id) { return dpp_d<0x130, 0xf, 0xf>(v, id); }

__device__ __forceinline__ double readlane_d(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}

}  // namespace
}  // namespace sq
