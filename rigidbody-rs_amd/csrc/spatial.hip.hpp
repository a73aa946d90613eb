// spatial.hip.hpp -- per-lane spatial algebra for the batched kernels (device only).
//
// One GPU lane owns one configuration; everything below is straight-line register
// arithmetic on 3-vectors, written with explicit FMAs so the instruction count is
// what the roofline in DESIGN.md assumes.  Conventions follow the reference:
//   spatial vectors are (rot, lin) pairs, Featherstone ordering (spatial.rs:137-149);
//   link pose T_i = (E_i, p_i), E_i = R_p,i * Rz(q_i)   (joint.rs:36-38, 48-50)
//   motion parent->child:  w' = E^T w,  v' = E^T (v - p x w)      (spatial.rs:110-116)
//   force  child->parent:  f' = E f,    n' = E n + p x (E f)      (spatial.rs:242-248
//                                                                  with Isometry::inverse)
//   rigid-body inertia (m, h = m c, I_o):  I*(w,v) = (I_o w + h x v,  m v - h x w)
//                                                                  (inertia.rs:107-117)
//   v x* f = (w x n + v x f,  w x f)                               (spatial.rs:129-134)
#pragma once

#if defined(__HIPCC_RTC__)
// hipRTC compiles this header for the model-specialised kernels (jit.cpp); it brings
// the HIP device builtins itself but not <cstdint>.
typedef unsigned int uint32_t;
typedef long long int64_t;
typedef unsigned long long uint64_t;
#else
#include <hip/hip_runtime.h>

#include <cstdint>
#endif

#include "layout.hpp"

// Per-configuration algebra is host+device: the same lane bodies serve the GPU kernels and
// the host single-configuration ABI (host_eval.cpp).  Functions that touch device memory
// spaces or GPU-only builtins (row access, LDS staging, hardware reciprocal) stay __device__.
#if defined(__HIPCC_RTC__)
#define RB_HD __device__ __forceinline__
#else
#define RB_HD __host__ __device__ __forceinline__
#endif

namespace rbamd {
namespace dev {

RB_HD float fmadd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
RB_HD double fmadd(double a, double b, double c) { return __builtin_fma(a, b, c); }

// Paired fp32 lanes (model-specialised fp32 kernels, tuning `pack`): a lane evaluates two
// configurations at once as a 2-wide vector, so every FMA/MUL/ADD of the recursion becomes
// one v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (FR3 RNEA: 646 VALU instructions per PAIR
// vs 586 per configuration).  It pays for the issue-/latency-bound forward dynamics (FR3:
// 28.0 vs 29.0-30.7 us; the same pairing as two scalar FMAs per operation: 33.7 us, DESIGN.md
// §4), not for the memory-bound RNEA.  Only sin/cos and 1/x stay per element; both halves run
// identical instruction sequences.
typedef float f2 __attribute__((ext_vector_type(2)));
RB_HD f2 fmadd(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <typename T>
struct V3 {
    T x, y, z;
};

template <typename T>
RB_HD V3<T> v3(T x, T y, T z) { return V3<T>{x, y, z}; }

// a x b
template <typename T>
RB_HD V3<T> cross(const V3<T> &a, const V3<T> &b) {
    return v3(fmadd(a.y, b.z, -a.z * b.y), fmadd(a.z, b.x, -a.x * b.z), fmadd(a.x, b.y, -a.y * b.x));
}

// acc + a x b
template <typename T>
RB_HD V3<T> cross_add(const V3<T> &acc, const V3<T> &a, const V3<T> &b) {
    return v3(fmadd(a.y, b.z, fmadd(-a.z, b.y, acc.x)), fmadd(a.z, b.x, fmadd(-a.x, b.z, acc.y)),
              fmadd(a.x, b.y, fmadd(-a.y, b.x, acc.z)));
}

// acc - a x b
template <typename T>
RB_HD V3<T> cross_sub(const V3<T> &acc, const V3<T> &a, const V3<T> &b) {
    return v3(fmadd(-a.y, b.z, fmadd(a.z, b.y, acc.x)), fmadd(-a.z, b.x, fmadd(a.x, b.z, acc.y)),
              fmadd(-a.x, b.y, fmadd(a.y, b.x, acc.z)));
}

// Row-major 3x3.
template <typename T>
struct M3 {
    T m[9];
};

// M x
template <typename T>
RB_HD V3<T> mul(const M3<T> &M, const V3<T> &x) {
    return v3(fmadd(M.m[0], x.x, fmadd(M.m[1], x.y, M.m[2] * x.z)),
              fmadd(M.m[3], x.x, fmadd(M.m[4], x.y, M.m[5] * x.z)),
              fmadd(M.m[6], x.x, fmadd(M.m[7], x.y, M.m[8] * x.z)));
}

// acc + M x
template <typename T>
RB_HD V3<T> mul_add(const V3<T> &acc, const M3<T> &M, const V3<T> &x) {
    return v3(fmadd(M.m[0], x.x, fmadd(M.m[1], x.y, fmadd(M.m[2], x.z, acc.x))),
              fmadd(M.m[3], x.x, fmadd(M.m[4], x.y, fmadd(M.m[5], x.z, acc.y))),
              fmadd(M.m[6], x.x, fmadd(M.m[7], x.y, fmadd(M.m[8], x.z, acc.z))));
}

// M^T x
template <typename T>
RB_HD V3<T> mul_t(const M3<T> &M, const V3<T> &x) {
    return v3(fmadd(M.m[0], x.x, fmadd(M.m[3], x.y, M.m[6] * x.z)),
              fmadd(M.m[1], x.x, fmadd(M.m[4], x.y, M.m[7] * x.z)),
              fmadd(M.m[2], x.x, fmadd(M.m[5], x.y, M.m[8] * x.z)));
}

// Symmetric 3x3: xx xy xz yy yz zz
template <typename T>
struct S3 {
    T xx, xy, xz, yy, yz, zz;
};

template <typename T>
RB_HD V3<T> mul(const S3<T> &S, const V3<T> &x) {
    return v3(fmadd(S.xx, x.x, fmadd(S.xy, x.y, S.xz * x.z)),
              fmadd(S.xy, x.x, fmadd(S.yy, x.y, S.yz * x.z)),
              fmadd(S.xz, x.x, fmadd(S.yz, x.y, S.zz * x.z)));
}

template <typename T>
RB_HD V3<T> mul_add(const V3<T> &acc, const S3<T> &S, const V3<T> &x) {
    return v3(fmadd(S.xx, x.x, fmadd(S.xy, x.y, fmadd(S.xz, x.z, acc.x))),
              fmadd(S.xy, x.x, fmadd(S.yy, x.y, fmadd(S.yz, x.z, acc.y))),
              fmadd(S.xz, x.x, fmadd(S.yz, x.y, fmadd(S.zz, x.z, acc.z))));
}

// Topology of the reference's Multibody (multibody.rs:32): a serial chain of revolute
// joints, parent(j) = j - 1.  The lane functions take a `Topo` policy; this one selects the
// tuned serial code, a model-specialised kernel of a tree model gets its own (jit.cpp,
// tree_body.hip.hpp).
struct SerialTopo {
    static constexpr bool kSerial = true;
    static constexpr int parent(int j) { return j - 1; }
    static constexpr bool prismatic(int) { return false; }
    static constexpr bool on_path(int) { return true; }  // every link is an ancestor of the last
};

// Per-link model constants.  Each workgroup first copies the packed block (layout.hpp,
// n * 24 scalars, <= 5.8 KB) from HBM/L2 into LDS (stage_model); every later read is a
// wave-uniform LDS broadcast, issued where the link is processed.  (Reading the block
// with scalar loads instead makes the compiler hoist all n*22 constants into SGPRs and
// spill them: 58 spills at fp32 / 224 at fp64 for the 7-DOF RNEA.)
template <typename T>
struct Link {
    M3<T> Rp;
    V3<T> p;
    T m;
    V3<T> h;
    S3<T> Io;
};

// Two-phase staging so a block's model fetch overlaps its first joint-value loads:
// fetch() issues the global loads of the packed block into registers, the caller then
// issues its own input loads, and commit() writes LDS and joins the block at a barrier
// that waits for LDS traffic only (lgkmcnt), not for the input loads in flight
// (__syncthreads() would add vmcnt(0) and serialise the two latencies).
template <typename T, int N, int BLOCK>
struct ModelStage {
    static constexpr int kElems = N * kLinkStride;
    static constexpr int K = (kElems + BLOCK - 1) / BLOCK;
    T v[K];
    __device__ __forceinline__ void fetch(const T *__restrict__ g) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = threadIdx.x + k * BLOCK;
            v[k] = i < kElems ? g[i] : T(0);
        }
    }
    __device__ __forceinline__ void commit(T *smem) const {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = threadIdx.x + k * BLOCK;
            if (i < kElems) smem[i] = v[k];
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
};

template <typename T, int N, int BLOCK>
__device__ __forceinline__ void stage_model(const T *__restrict__ mdl, T *smem) {
    ModelStage<T, N, BLOCK> st;
    st.fetch(mdl);
    st.commit(smem);
}

// Model-specialised kernels (RB_OPAQUE_CONSTS, jit.cpp): a compile-time model value that is
// not 0 or +-1 is pinned to its use site through an SGPR (s_mov per use, scalar pipe),
// so a runtime loop around the dynamics (the rollout) does not hoist ~70 literals into
// registers for its whole lifetime.  The structural 0 / +-1 entries still fold away.
#ifndef RB_OPAQUE_CONSTS
#define RB_OPAQUE_CONSTS 0
#endif
template <typename T>
RB_HD T mconst(T v) {
    if constexpr (RB_OPAQUE_CONSTS != 0) {
        if (__builtin_constant_p(v) && v != T(0) && v != T(1) && v != T(-1)) asm volatile("" : "+s"(v));
    }
    return v;
}
RB_HD f2 mconst(f2 v) {
    // Paired kernels pin only under a runtime loop (the paired rollout): one SGPR per
    // constant, which v_pk_fma broadcasts to both halves.
    if constexpr (RB_OPAQUE_CONSTS != 0) {
        if (__builtin_constant_p(v.x) && v.x != 0.0f && v.x != 1.0f && v.x != -1.0f) {
            float c = v.x;
            asm volatile("" : "+s"(c));
            return f2{c, c};
        }
    }
    return v;
}

template <typename T>
RB_HD Link<T> load_link(const T *__restrict__ mdl, int i) {
    const T *c = mdl + i * kLinkStride;
    Link<T> L;
#pragma unroll
    for (int k = 0; k < 9; ++k) L.Rp.m[k] = mconst(c[kE0 + k]);
    L.p = v3(mconst(c[kP + 0]), mconst(c[kP + 1]), mconst(c[kP + 2]));
    L.m = mconst(c[kM]);
    L.h = v3(mconst(c[kH + 0]), mconst(c[kH + 1]), mconst(c[kH + 2]));
    L.Io = S3<T>{mconst(c[kIo + 0]), mconst(c[kIo + 1]), mconst(c[kIo + 2]),
                 mconst(c[kIo + 3]), mconst(c[kIo + 4]), mconst(c[kIo + 5])};
    return L;
}

// E = R_p * Rz(q): columns 0/1 mix with (cos, sin), column 2 is R_p's.
template <typename T>
RB_HD M3<T> joint_rotation(const M3<T> &Rp, T c, T s) {
    M3<T> E;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const T a = Rp.m[3 * r + 0], b = Rp.m[3 * r + 1];
        E.m[3 * r + 0] = fmadd(a, c, b * s);
        E.m[3 * r + 1] = fmadd(b, c, -a * s);
        E.m[3 * r + 2] = Rp.m[3 * r + 2];
    }
    return E;
}

// Rigid-body inertia times a motion vector (inertia.rs:107-117); returns (rot, lin).
template <typename T>
RB_HD void inertia_mul(const Link<T> &L, const V3<T> &w, const V3<T> &v,
                                            V3<T> &n, V3<T> &f) {
    n = cross_add(mul(L.Io, w), L.h, v);                     // I_o w + h x v
    f = cross_sub(v3(L.m * v.x, L.m * v.y, L.m * v.z), L.h, w);  // m v - h x w
}

// Link force f = I a + v x* (I v) (inertia.rs:107-117, spatial.rs:129-134) for a link moving
// with (w, v) and accelerating with (aw, av), both spatial, in link coordinates.
// Model-specialised kernels of serial chains (RB_COM_FORM, jit.cpp) evaluate it as the
// Newton-Euler equations about the centre of mass c with the COM inertia Ic (per-link
// constants rb_com[9j..] = c, Ic, computed on the host in fp64 from m, h, I_o):
//   vc = v + w x c,  ac = a + aw x c,  f = m (ac + w x vc),  n = Ic aw + w x (Ic w) + c x f
// -- the same quantity (f is m times the COM's classical acceleration, n Euler's equation
// moved to the link origin) in 51 instead of 66 FMAs.
#ifndef RB_COM_FORM
#define RB_COM_FORM 0
#endif
#if RB_COM_FORM
template <typename T>
RB_HD T com_k(double x) { return T(x); }
template <>
RB_HD f2 com_k<f2>(double x) { return f2{(float)x, (float)x}; }
template <typename T>
RB_HD void link_force(const Link<T> &L, int j, const V3<T> &w, const V3<T> &v, const V3<T> &aw, const V3<T> &av,
                      V3<T> &fn, V3<T> &ff) {
    const double *k = rb_com + 9 * j;
    const V3<T> c = v3(com_k<T>(k[0]), com_k<T>(k[1]), com_k<T>(k[2]));
    const S3<T> Ic{com_k<T>(k[3]), com_k<T>(k[4]), com_k<T>(k[5]), com_k<T>(k[6]), com_k<T>(k[7]), com_k<T>(k[8])};
    const V3<T> vc = cross_add(v, w, c);
    const V3<T> g = cross_add(cross_add(av, aw, c), w, vc);
    ff = v3(L.m * g.x, L.m * g.y, L.m * g.z);
    fn = cross_add(cross_add(mul(Ic, aw), w, mul(Ic, w)), c, ff);
}
// The same wrench with the force left unscaled: g = f / m is returned and n uses c x f = h x g
// (h = m c).  The forward dynamics' bias sweep (fdh_body.hip.hpp) multiplies by m in its backward
// sweep, where the product takes the child's transmitted force as its FMA addend.
template <typename T>
RB_HD void link_force_g(const Link<T> &L, int j, const V3<T> &w, const V3<T> &v, const V3<T> &aw, const V3<T> &av,
                        V3<T> &fn, V3<T> &g) {
    const double *k = rb_com + 9 * j;
    const V3<T> c = v3(com_k<T>(k[0]), com_k<T>(k[1]), com_k<T>(k[2]));
    const S3<T> Ic{com_k<T>(k[3]), com_k<T>(k[4]), com_k<T>(k[5]), com_k<T>(k[6]), com_k<T>(k[7]), com_k<T>(k[8])};
    const V3<T> vc = cross_add(v, w, c);
    g = cross_add(cross_add(av, aw, c), w, vc);
    fn = cross_add(cross_add(mul(Ic, aw), w, mul(Ic, w)), L.h, g);
}
#else
template <typename T>
RB_HD void link_force(const Link<T> &L, int, const V3<T> &w, const V3<T> &v, const V3<T> &aw, const V3<T> &av,
                      V3<T> &fn, V3<T> &ff) {
    V3<T> In, If, An, Af;
    inertia_mul(L, w, v, In, If);
    inertia_mul(L, aw, av, An, Af);
    ff = cross_add(Af, w, If);
    fn = cross_add(cross_add(An, w, In), v, If);
}
#endif

// SoA row access: uniform row base (SGPRs) + a 32-bit per-lane byte offset, so loads and
// stores use the global_load/store saddr form with one shared offset VGPR instead of a
// 64-bit address per access.  Callers keep b * sizeof(T) < 2^32 (per-launch batch cap).
// RB_NT (set by the hipRTC source, jit.cpp): bit 0 non-temporal row loads, bit 1
// non-temporal row stores -- every input/output element is touched exactly once.
#ifndef RB_VARIANT
#define RB_VARIANT 0
#endif
#ifndef RB_NT
#define RB_NT 0
#endif
// Row pointers are typed global (address_space(1)): from a generic pointer the compiler
// strength-reduces consecutive row addresses into chained 64-bit per-lane VGPR adds (68 of
// them in the FR3 RNEA kernel), which costs VALU and VGPRs and -- when it reuses a pending
// load's destination register as an address half -- a full memory-latency wait in the middle
// of the load burst.  Typed global, every access is the saddr form: uniform 64-bit row base
// in SGPRs + the lane's 32-bit byte offset.  (RB_VARIANT bit 6 restores the generic form
// for A/B measurements.)
template <typename T>
using gptr = __attribute__((address_space(1))) T *;

// NTL = false: a temporal load whatever RB_NT says (a row the lane will read again).
template <typename T, bool NTL = (RB_NT & 1) != 0>
__device__ __forceinline__ T ld_row(const T *__restrict__ base, int64_t row, uint32_t off) {
    if constexpr (!NTL) {
        gptr<const T> p = (gptr<const T>)((gptr<const char>)(base + row) + off);
        return *p;
    } else if constexpr ((RB_VARIANT & 64) != 0) {
        const T *p = reinterpret_cast<const T *>(reinterpret_cast<const char *>(base + row) + off);
        if constexpr ((RB_NT & 1) != 0) return __builtin_nontemporal_load(p);
        return *p;
    } else {
        gptr<const T> p = (gptr<const T>)((gptr<const char>)(base + row) + off);
        if constexpr ((RB_NT & 1) != 0) return __builtin_nontemporal_load(p);
        return *p;
    }
}
template <typename T>
__device__ __forceinline__ void st_row(T *__restrict__ base, int64_t row, uint32_t off, T v) {
    if constexpr ((RB_VARIANT & 64) != 0) {
        T *p = reinterpret_cast<T *>(reinterpret_cast<char *>(base + row) + off);
        if constexpr ((RB_NT & 2) != 0) {
            __builtin_nontemporal_store(v, p);
        } else {
            *p = v;
        }
    } else {
        gptr<T> p = (gptr<T>)((gptr<char>)(base + row) + off);
        if constexpr ((RB_NT & 2) != 0) {
            __builtin_nontemporal_store(v, p);
        } else {
            *p = v;
        }
    }
}

// Compiler-only fence: forces per-link constants to be re-read from LDS in a later
// sweep instead of being kept live in VGPRs across the whole chain.
RB_HD void reload_fence() { asm volatile("" ::: "memory"); }

// Stage markers for the per-stage instruction audit (tools/fd_stages.py): an assembler comment
// fenced by scheduling barriers, so the ISA splits where one stage ends.  Off in the product.
#ifndef RB_STAGE_MARKS
#define RB_STAGE_MARKS 0
#endif
#if defined(RB_STAGE)
// a host tool's own stage hook (tools/opcount.py)
#elif RB_STAGE_MARKS
#define RB_STAGE(name)                                       \
    do {                                                     \
        __builtin_amdgcn_sched_barrier(0);                   \
        asm volatile("; rb_stage " name ::: "memory");       \
        __builtin_amdgcn_sched_barrier(0);                   \
    } while (0)
#else
#define RB_STAGE(name) \
    do {               \
    } while (0)
#endif


// ---------------------------------------------------------------------------- sincos
// Joint angles need sin/cos once per link.  The ROCm device-library sincos carries a
// Payne-Hanek branch for huge arguments that inflates every unrolled kernel's register
// footprint (fp64 7-DOF RNEA: 256 VGPR + 123 AGPR, 1 wave/SIMD).  These are
// branch-free: Cody-Waite reduction by pi/2 with a 3-term FMA split, then the fdlibm
// __kernel_sin/__kernel_cos minimax polynomials on |r| <= pi/4 (<= 1 ulp for
// |x| < 2^20 rad -- far beyond any joint angle).  FAST=true (fp32 only) uses the
// hardware v_sin_f32/v_cos_f32.
RB_HD void sincos_cw(double x, double &s, double &c) {
#if !defined(__HIP_DEVICE_COMPILE__) && !defined(__HIPCC_RTC__)
    // host single-configuration path: past the reduction's exact range (and for NaN / Inf) the
    // C library, as the reference's from_scaled_axis -- any finite angle is exact there
    if (!(__builtin_fabs(x) < 0x1p45)) {
        s = __builtin_sin(x);
        c = __builtin_cos(x);
        return;
    }
#endif
    const double k = __builtin_rint(x * 6.36619772367581382433e-01);  // 2/pi
    double r = __builtin_fma(-k, 1.57079632679489655800e+00, x);      // pi/2 hi
    r = __builtin_fma(-k, 6.12323399573676603587e-17, r);              // pi/2 mid
    r = __builtin_fma(-k, -1.49738490485916983e-33, r);                // pi/2 lo
    const double z = r * r;
    const double v = z * r;
    const double ps = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                          1.58969099521155010221e-10, -2.50507602534068634195e-08),
                          2.75573137070700676789e-06), -1.98412698298579493134e-04),
                          8.33333333332248946124e-03);
    const double sr = __builtin_fma(v, __builtin_fma(z, ps, -1.66666666666666324348e-01), r);
    const double pc = z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                          __builtin_fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                          -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                          -1.38888888888741095749e-03), 4.16666666666666019037e-02);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * pc);
    const int q = (int)(long long)k & 3;
    const double ss = (q & 1) ? cr : sr;
    const double cc = (q & 1) ? sr : cr;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}

RB_HD void sincos_cw(float x, float &s, float &c) {
    const float k = __builtin_rintf(x * 6.3661977236e-01f);
    float r = __builtin_fmaf(-k, 1.57079637e+00f, x);
    r = __builtin_fmaf(-k, -4.37113883e-08f, r);
    r = __builtin_fmaf(-k, -1.71512451e-15f, r);
    const float z = r * r;
    const float sr = __builtin_fmaf(z * r, __builtin_fmaf(z, __builtin_fmaf(z, -1.9515295891e-4f,
                                    8.3321608736e-3f), -1.6666654611e-1f), r);
    const float cr = __builtin_fmaf(z * z, __builtin_fmaf(z, __builtin_fmaf(z, 2.443315711809948e-5f,
                                    -1.388731625493765e-3f), 4.166664568298827e-2f), __builtin_fmaf(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    const float ss = (q & 1) ? cr : sr;
    const float cc = (q & 1) ? sr : cr;
    s = (q & 2) ? -ss : ss;
    c = ((q + 1) & 2) ? -cc : cc;
}

// FAST fp32: the hardware v_sin_f32 / v_cos_f32, which take revolutions.  The angle is reduced
// to revolutions exactly first: k = rint(x / 2pi) from the 1.5 * 2^23 shifter, then
// u = x (1/2pi)_hi - k + x (1/2pi)_lo with the first two terms in one FMA (x (1/2pi)_hi and k
// agree in their leading bits, so the FMA's single rounding leaves u accurate to its own ulp).
// A plain x * (1/2pi) carries a relative error of 2^-24 into the revolutions -- 6e-6 rad at
// |x| = 100 -- and past 256 revolutions the instruction's input range is exceeded; the reduced
// form keeps |q| <= pi accuracy for every |x| < 2^22 * 2 pi (the supported range is 2^22 rad,
// InputGuard).  4 VALU per angle instead of 1 (packed pairs: 4 v_pk per pair).
constexpr float kInv2PiHi = 0x1.45f306p-3f, kInv2PiLo = 0x1.b93910p-28f;  // 1/2pi = hi + lo + 7e-17
constexpr float kRevShifter = 0x1.8p23f;                                 // 1.5 * 2^23
RB_HD void sincos_hw(float x, float &s, float &c) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr ((RB_VARIANT & 4096) != 0) {  // A/B only: the unreduced x * (1/2pi) of round 4
        s = __builtin_amdgcn_sinf(x * kInv2PiHi);
        c = __builtin_amdgcn_cosf(x * kInv2PiHi);
        return;
    }
    const float k = __builtin_fmaf(x, kInv2PiHi, kRevShifter) - kRevShifter;
    const float u = __builtin_fmaf(x, kInv2PiLo, __builtin_fmaf(x, kInv2PiHi, -k));
    s = __builtin_amdgcn_sinf(u);
    c = __builtin_amdgcn_cosf(u);
#else
    sincos_cw(x, s, c);
#endif
}
RB_HD void sincos_hw(f2 x, f2 &s, f2 &c) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr ((RB_VARIANT & 4096) != 0) {
        float s0, c0, s1, c1;
        sincos_hw(x.x, s0, c0);
        sincos_hw(x.y, s1, c1);
        s = f2{s0, s1};
        c = f2{c0, c1};
        return;
    }
    const f2 hi = f2{kInv2PiHi, kInv2PiHi}, lo = f2{kInv2PiLo, kInv2PiLo}, sh = f2{kRevShifter, kRevShifter};
    const f2 k = fmadd(x, hi, sh) - sh;
    const f2 u = fmadd(x, lo, fmadd(x, hi, -k));
    s = f2{__builtin_amdgcn_sinf(u.x), __builtin_amdgcn_sinf(u.y)};
    c = f2{__builtin_amdgcn_cosf(u.x), __builtin_amdgcn_cosf(u.y)};
#else
    float s0, c0, s1, c1;
    sincos_cw(x.x, s0, c0);
    sincos_cw(x.y, s1, c1);
    s = f2{s0, s1};
    c = f2{c0, c1};
#endif
}

template <bool FAST>
RB_HD void sin_cos(float x, float &s, float &c) {
    if constexpr (FAST) {
        sincos_hw(x, s, c);
    } else {
        sincos_cw(x, s, c);
    }
}
// Table-assisted fp64 sincos for the model-specialised fp64 kernels (RB_SINCOS_TAB, set by
// jit.cpp): x = k pi/128 + r with |r| <= pi/256, (cos, sin)(k pi/128) from a 256-entry LDS table
// the block copies once (sctab_init; the entries rb_sctab_src[2k], [2k+1] are computed on the host
// in long double, quadrant points exact, and compiled into the hipRTC source), then a degree-5
// minimax sine (leading term r exact, relative error <= 2.7e-17 on |r| <= 1.002 pi/256) and a
// degree-6 Taylor cosine (truncation 1.3e-20), and one angle-addition step.  k comes from the
// 1.5 * 2^52 shifter: fma(x, 128/pi, 1.5 * 2^52) rounds x 128/pi to the nearest integer and
// leaves it, two's complement, in the low word -- the table index without a conversion.
// 18 VALU instructions per angle (the previous pi/32 table: 23, plus ~65 on the block's first
// wave to fill it); max error 2.8 ulp over |x| <= 100 (host emulation, 2e7 samples; the pi/32
// table: 2.7).
#ifndef RB_SINCOS_TAB
#define RB_SINCOS_TAB 0
#endif
#if RB_SINCOS_TAB
struct alignas(16) SinCosEntry {
    double c, s;
};
__shared__ SinCosEntry rb_sctab[256];

// Every wave of the block must call this before any sin_cos(double) (it ends in a barrier);
// any block size (one entry per thread for the 256-thread blocks every JIT kernel uses).
__device__ __forceinline__ void sctab_init() {
    for (uint32_t t = threadIdx.x; t < 256u; t += blockDim.x)
        rb_sctab[t] = SinCosEntry{rb_sctab_src[2 * t], rb_sctab_src[2 * t + 1]};
    __syncthreads();
}

__device__ __forceinline__ void sincos_tab(double x, double &s, double &c) {
    const double shifter = 6755399441055744.0;                      // 1.5 * 2^52
    const double t = __builtin_fma(x, 4.074366543152521e+01, shifter);  // 128/pi
    const double k = t - shifter;
    const uint32_t ki = (uint32_t)__builtin_bit_cast(unsigned long long, t) & 255u;
    // two-term Cody-Waite: pi/128 - (hi + mid) = -2.3e-35, which over the supported |x| < 2^41
    // (|k| < 2^46.4, InputGuard) moves r by < 2.2e-21, 1/1000 of an ulp of r -- a third FMA
    // with the lo term buys nothing there
    double r = __builtin_fma(-k, 2.454369260617026e-02, x);         // pi/128 hi
    r = __builtin_fma(-k, 9.567553118338697e-19, r);                 // pi/128 mid
    const SinCosEntry e = rb_sctab[ki];
    const double z = r * r;
    const double sr = __builtin_fma(r * z, __builtin_fma(z, 8.333291563954032e-03, -1.666666666647126e-01), r);
    const double cr = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, -1.3888888888888889e-03,
                          4.1666666666666664e-02), -0.5), 1.0);
    s = __builtin_fma(e.s, cr, e.c * sr);
    c = __builtin_fma(e.c, cr, -(e.s * sr));
}
#endif

template <bool FAST>
RB_HD void sin_cos(double x, double &s, double &c) {
#if RB_SINCOS_TAB
    sincos_tab(x, s, c);
#else
    sincos_cw(x, s, c);
#endif
}
template <bool FAST>
RB_HD void sin_cos(f2 x, f2 &s, f2 &c) {
    if constexpr (FAST) {
        sincos_hw(x, s, c);
        return;
    }
    float s0, c0, s1, c1;
    sin_cos<FAST>(x.x, s0, c0);
    sin_cos<FAST>(x.y, s1, c1);
    s = f2{s0, s1};
    c = f2{c0, c1};
}

// 1/x for the ABA's joint-space inertia D > 0 (normal range).  The IEEE division the
// compiler emits is ~10 instructions (div_scale x2, rcp, 4 FMAs, div_fmas, div_fixup);
// the hardware reciprocal is 1 ulp in fp32.  In fp64 v_rcp_f64 is good to 4.6e-8 relative and
// one Newton step to 2.2e-15 (~10 ulp; two steps: correctly rounded), measured over 2^22 inputs
// across 2^-60..2^61 (tools/probe_rcp.hip, profiles/r04/ab/probe_rcp.log) -- far inside the
// forward dynamics' 1e-8 tolerance, 14 VALU fewer per FR3 evaluation (jit_variant bit 1024 = the
// second step, A/B only).
__device__ __forceinline__ float recip(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
    if constexpr ((RB_VARIANT & 1024) != 0) r = __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
    return r;
}
__device__ __forceinline__ f2 recip(f2 x) { return f2{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)}; }

// ---------------------------------------------------------------------------- input guard
// The batched kernels' input domain (include/rigidbody_batch.h "Input domain"): every input
// finite and every revolute joint angle |q_j| < 2^41 rad (fp64) / 2^22 rad (fp32) -- inside the
// exact range of each sincos reduction above.  A configuration outside it gets NaN in every
// output.  The reference propagates NaN / Inf through its arithmetic (multibody.rs:111-174), but
// the model-specialised kernels cannot lean on propagation: they compile under
// -ffinite-math-only with the model's structural zeros folded, so FR3's torques, say, never
// read q_0 (a rotation about the gravity axis) and a NaN there would leave them finite.  So the
// kernels check, with arithmetic on an opaque zero z the compiler can neither fold nor reason
// about: acc = sum_j v(x_j) z is +-0 while every input is finite and NaN once one is not;
// angles are scaled by 2^128 / limit first, so |q| >= limit overflows to Inf.  Every output
// leaves as y + acc.  The check runs in fp32 (one VGPR, half the issue cost of fp64): v(x) is x,
// or for fp64 inputs the high word of x read as a float -- sign, the top 8 of the 11 exponent
// bits, 23 mantissa bits -- which is Inf / NaN exactly when x's exponent is >= 0x7f8 (x is
// NaN, Inf, or |x| >= 2^1017) and >= 2^6 exactly when |x| >= 2^41.  Cost per configuration:
// one FMA per input, one more per angle, one add per output (packed pairs: v_pk for both).
// On the host (the single-configuration ABI) angles are checked for Inf / NaN only: sincos_cw
// falls back to the C library past 2^45, so every finite angle is in range there, as in the
// reference.
//
// Out of the optimizer's reach.  The model-specialised kernels compile under
// -ffinite-math-only, where LLVM may treat the NaN of an nnan operation, or the Inf of an ninf
// one, as poison -- and may fold a bit test on such a value (e.g. into is.fpclass of a value
// "known" not to be NaN).  So on the device every step of the check is an instruction the
// compiler cannot see into: the scaled angle (v_mul), the accumulation (v_fma, z an SGPR) and
// the output add (fp32) are inline assembly, and fp64 outputs test acc's bits shifted by an asm
// v_lshlrev (an integer of unknown origin, not a bitcast of a float).  Same instructions, same
// count as the plain arithmetic; each carries the assembly comment "rb_guard" so a test can
// count them in the ISA (tests/test_boundary.py).
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
#define RB_GUARD_ASM 1
#else
#define RB_GUARD_ASM 0
#endif
RB_HD float guard_view(float x) { return x; }
RB_HD f2 guard_view(f2 x) { return x; }
RB_HD float guard_view(double x) {
    return __builtin_bit_cast(float, (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32));
}
RB_HD float angle_scale(double) { return 0x1p122f; }  // high word >= 2^6 (|q| >= 2^41) -> Inf
RB_HD float angle_scale(float) { return 0x1p106f; }   // |q| >= 2^22 -> Inf
RB_HD f2 angle_scale(f2) { return f2{0x1p106f, 0x1p106f}; }
RB_HD float guard_acc(double) { return 0.0f; }
RB_HD float guard_acc(float) { return 0.0f; }
RB_HD f2 guard_acc(f2) { return f2{0.0f, 0.0f}; }

// acc + v z
RB_HD float guard_fma(float v, float z, float acc) {
#if RB_GUARD_ASM
    asm("v_fma_f32 %0, %1, %2, %0 ; rb_guard" : "+v"(acc) : "v"(v), "s"(z));
    return acc;
#else
    return __builtin_fmaf(v, z, acc);
#endif
}
RB_HD f2 guard_fma(f2 v, f2 z, f2 acc) {
#if RB_GUARD_ASM
    asm("v_pk_fma_f32 %0, %1, %2, %0 ; rb_guard" : "+v"(acc) : "v"(v), "s"(z));
    return acc;
#else
    return fmadd(v, z, acc);
#endif
}
// v * scale (Inf past the angle bound)
RB_HD float guard_scale(float v, float sc) {
#if RB_GUARD_ASM
    float r;  // a fresh register: v (the angle's high word) lives on for the sincos
    asm("v_mul_f32 %0, %1, %2 ; rb_guard" : "=v"(r) : "s"(sc), "v"(v));
    return r;
#else
    return v * sc;
#endif
}
RB_HD f2 guard_scale(f2 v, f2 sc) {
#if RB_GUARD_ASM
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 ; rb_guard" : "=v"(r) : "s"(sc), "v"(v));
    return r;
#else
    return v * sc;
#endif
}
// y + acc
RB_HD float guard_add(float y, float acc) {
#if RB_GUARD_ASM
    float r;
    asm("v_add_f32 %0, %1, %2 ; rb_guard" : "=v"(r) : "v"(acc), "v"(y));
    return r;
#else
    return y + acc;
#endif
}
RB_HD f2 guard_add(f2 y, f2 acc) {
#if RB_GUARD_ASM
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 ; rb_guard" : "=v"(r) : "v"(acc), "v"(y));
    return r;
#else
    return y + acc;
#endif
}
// acc's bits shifted left by one (the sign dropped) as an integer the compiler knows nothing
// about: the shift the NaN test needs anyway, issued as asm, so the test below cannot be
// recognised as an is-NaN test of a float (which no-nans-fp-math would fold to false).
RB_HD uint32_t guard_bits2(float acc) {
#if RB_GUARD_ASM
    uint32_t t;
    asm("v_lshlrev_b32 %0, 1, %1 ; rb_guard" : "=v"(t) : "v"(acc));
    return t;
#else
    return __builtin_bit_cast(uint32_t, acc) << 1;
#endif
}

template <typename T>
struct InputGuard {
    using A = decltype(guard_acc(T()));
    A z, acc;
    RB_HD InputGuard() : z(guard_acc(T())) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
        asm("" : "+s"(z));
#endif
        acc = z;
    }
    // RB_VARIANT bit 2048 (A/B only): no checks -- the round-4 kernels' arithmetic
    static constexpr bool kOff = (RB_VARIANT & 2048) != 0;
    RB_HD void val(T x) {
        if constexpr (!kOff) acc = guard_fma(guard_view(x), z, acc);
    }
    RB_HD void angle(T x) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC_RTC__)
        // bit 8192 (A/B only): no angle checks (rows the dynamics never read stay unread)
        if constexpr (!kOff && (RB_VARIANT & 8192) == 0)
            acc = guard_fma(guard_scale(guard_view(x), angle_scale(x)), z, acc);
#else
        val(x);
#endif
    }
    template <int N>
    RB_HD void vals(const T (&x)[N]) {
#pragma unroll
        for (int j = 0; j < N; ++j) val(x[j]);
    }
    // joint positions: angles of revolute joints, displacements of prismatic ones
    template <typename Topo, int N>
    RB_HD void joints(const T (&q)[N]) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (Topo::prismatic(j))
                val(q[j]);
            else
                angle(q[j]);
        }
    }
    // fp32 outputs: y + acc.  fp64 outputs: the high word OR-ed with 0x7ff80000 (a quiet NaN
    // whatever the rest) when acc is NaN -- one 32-bit integer op per output instead of an fp64
    // add, and no fp64 copy of acc held across the backward sweep (fp64 FR3 pair: 127 instead
    // of 129 VGPRs, the 4th wave per SIMD).  acc is +-0 or NaN: NaN iff (bits << 1) > 0xff000000.
    RB_HD T out(T y) const {
        if constexpr (kOff) {
            return y;
        } else if constexpr (__is_same(T, double)) {
            const uint32_t m = guard_bits2(acc) > 0xff000000u ? 0x7ff80000u : 0u;
            return __builtin_bit_cast(T, __builtin_bit_cast(uint64_t, y) | ((uint64_t)m << 32));
        } else {
            return guard_add(y, acc);
        }
    }
};

// Paired-lane row access: one configuration from each of two batch blocks.  Both halves
// use the saddr form off ONE wave-uniform base (the pair's first block, element oA): the
// first at the lane's byte offset offA, the second at offB = offA + the block stride in bytes
// (or offA itself when the second configuration is past B) -- per-lane 32-bit offsets, no
// 64-bit address arithmetic per row (a per-lane second base cost 2 v_lshl_add_u64 per row).
__device__ __forceinline__ f2 ld_row2(const float *__restrict__ base, int64_t row, uint32_t offA, uint32_t offB) {
    return f2{ld_row(base, row, offA), ld_row(base, row, offB)};
}
__device__ __forceinline__ void st_row2(float *__restrict__ base, int64_t row, uint32_t offA, uint32_t offB, f2 v) {
    st_row(base, row, offA, v.x);
    st_row(base, row, offB, v.y);
}

}  // namespace dev
}  // namespace rbamd
