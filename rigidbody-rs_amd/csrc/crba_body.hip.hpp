// crba_body.hip.hpp -- per-lane joint-space mass matrix (device).  Multibody::crba
// (multibody.rs:155-174): composite inertia leaf->root; column i of H from F = Ic_i S
// carried to the root.  Output follows the ABI: element e = row + n*col of the n x n
// column-major matrix, H[j + n*i] for j <= i, strictly-lower entries exact zeros.
#pragma once

#include "tree_body.hip.hpp"

namespace rbamd {
namespace dev {

// The recursion on given joint (cos, sin): also the mass-matrix stage of the forward dynamics
// (fdh_body.hip.hpp), which has them from its bias-torque sweep.
template <typename T, int N, typename Out>
RB_HD void crba_core(const T *mdl, const T (&cs)[N], const T (&sn)[N], Out &&out) {
    RigidI<T> Ic = rigid_of(load_link(mdl, N - 1));  // composite rigid body (artinertia.hip.hpp)
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        reload_fence();
        out(i + N * i, Ic.Io.zz);  // get_rotz, inertia.rs:91-93
#pragma unroll
        for (int r = i + 1; r < N; ++r) out(r + N * i, T(0));
        // F = Ic S, S = rot z:  n = I_o e_z,  f = -h x e_z = (-h.y, h.x, 0)
        V3<T> Fn = v3(Ic.Io.xz, Ic.Io.yz, Ic.Io.zz);
        V3<T> Ff = v3(-Ic.h.y, Ic.h.x, T(0));
#pragma unroll
        for (int j = i - 1; j >= 0; --j) {
            const Link<T> L = load_link(mdl, j + 1);
            const M3<T> E = joint_rotation(L.Rp, cs[j + 1], sn[j + 1]);
            const V3<T> fl = mul(E, Ff);
            Fn = cross_add(mul(E, Fn), L.p, fl);
            Ff = fl;
            out(j + N * i, Fn.z);
        }
        if (i > 0) {
            RB_STAGE("crba_composite");
            const Link<T> L = load_link(mdl, i);
            if constexpr (RB_SPLIT_ROT != 0 && RB_OPAQUE_CONSTS == 0) {
                Ic = rigid_to_parent_add(L.Rp, cs[i], sn[i], L.p, Ic, load_link(mdl, i - 1));
            } else {
                const M3<T> E = joint_rotation(L.Rp, cs[i], sn[i]);
                Ic = rigid_to_parent(L.Rp, cs[i], sn[i], E, L.p, Ic);
                add_rigid(Ic, load_link(mdl, i - 1));
            }
            RB_STAGE("crba_columns");
        }
    }
}

template <typename T, int N, bool FAST, typename Out>
RB_HD void crba_eval(const T *mdl, const T (&qv)[N], Out &&out) {
    InputGuard<T> gd;  // out-of-domain configurations: NaN upper triangle (spatial.hip.hpp)
    gd.template joints<SerialTopo>(qv);
    T cs[N], sn[N];
#pragma unroll
    for (int j = 0; j < N; ++j) sin_cos<FAST>(qv[j], sn[j], cs[j]);
    // strictly-lower entries (row > col) stay the ABI's exact zeros
    crba_core<T, N>(mdl, cs, sn, [&](int e, T v) { out(e, e % N <= e / N ? gd.out(v) : v); });
}

template <typename T, int N, bool FAST, typename Topo = SerialTopo>
__device__ __forceinline__ void crba_lane(const T *mdl, const T *__restrict__ q, T *__restrict__ H, uint32_t b,
                                          int64_t ld) {
    const uint32_t off = b * (uint32_t)sizeof(T);
    T qv[N];
#pragma unroll
    for (int j = 0; j < N; ++j) qv[j] = ld_row(q, j * ld, off);
    if constexpr (Topo::kSerial)
        crba_eval<T, N, FAST>(mdl, qv, [&](int e, T v) { st_row(H, e * ld, off, v); });
    else
        crba_eval_tree<T, N, FAST, Topo>(mdl, qv, [&](int e, T v) { st_row(H, e * ld, off, v); });
}

}  // namespace dev
}  // namespace rbamd
