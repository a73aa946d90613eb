// crba_body.hip.hpp -- per-lane joint-space mass matrix (device).  Multibody::crba
// (multibody.rs:155-174): composite inertia leaf->root; column i of H from F = Ic_i S
// carried to the root.  Output follows the ABI: element e = row + n*col of the n x n
// column-major matrix, H[j + n*i] for j <= i, strictly-lower entries exact zeros.
#pragma once

#include "tree_body.hip.hpp"

namespace rbamd {
namespace dev {

template <typename T, int N, bool FAST, typename Out>
RB_HD void crba_eval(const T *mdl, const T (&qv)[N], Out &&out) {
    T cs[N], sn[N];
#pragma unroll
    for (int j = 0; j < N; ++j) sin_cos<FAST>(qv[j], sn[j], cs[j]);

    ArtI<T> Ic = rigid_inertia(load_link(mdl, N - 1));
#pragma unroll
    for (int i = N - 1; i >= 0; --i) {
        reload_fence();
        out(i + N * i, Ic.A.zz);  // get_rotz, inertia.rs:91-93
#pragma unroll
        for (int r = i + 1; r < N; ++r) out(r + N * i, T(0));
        V3<T> Fn = v3(Ic.A.xz, Ic.A.yz, Ic.A.zz);
        V3<T> Ff = v3(Ic.B.m[6], Ic.B.m[7], Ic.B.m[8]);
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
            const Link<T> L = load_link(mdl, i);
            const M3<T> E = joint_rotation(L.Rp, cs[i], sn[i]);
            if constexpr (RB_SPLIT_ROT != 0)
                Ic = to_parent_split(L.Rp, cs[i], sn[i], E, L.p, Ic);
            else
                Ic = to_parent(E, L.p, Ic);
            add_rigid(Ic, load_link(mdl, i - 1));
        }
    }
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
