// dofs.cpp -- the DOF values the kernels are instantiated for.
#include "dofs.hpp"
#include "kernels.hpp"

namespace rbamd {

int supported_dofs(int *out, int cap) {
    static const int dofs[] = {
#define RB_LIST(N) N,
        RB_FOR_EACH_DOF(RB_LIST)
#undef RB_LIST
    };
    int n = (int)(sizeof(dofs) / sizeof(dofs[0]));
    for (int i = 0; i < n && i < cap; ++i) out[i] = dofs[i];
    return n;
}

bool dof_supported(int n) {
    switch (n) {
#define RB_CASE(N) case N:
        RB_FOR_EACH_DOF(RB_CASE)
#undef RB_CASE
        return true;
        default:
            return false;
    }
}

}  // namespace rbamd
