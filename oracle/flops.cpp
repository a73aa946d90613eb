// flops.cpp -- TEST INFRASTRUCTURE ONLY: the op-counting build of oracle.c.
//
// Compiles the unmodified fp64 restatement of the reference (oracle.c: multibody.rs:111-174,
// spatial.rs, inertia.rs, joint.rs with nalgebra's quaternion arithmetic) with `double` replaced
// by FlopD, a one-double struct whose arithmetic operators count what they execute.  The result
// pins the algorithmic operation count of the reference's own formulation per evaluation
// (SURVEY §8(d) "pin it by an op-counting build of the CPU oracle"), which bench.py reports as
// roofline.valu.flops_per_eval_ref.  FlopD has the layout of a double, so the model struct and
// every array argument are binary-compatible with liboracle.so's: the same ctypes calls drive
// either library (oracle/oracle.py op_counts).
//
// Counted: + - * / (one each), sqrt / sin / cos / acos (separately, one each).  Not counted:
// negation, comparisons, copies (nalgebra's are free too).
#include <cfloat>
#include <cmath>
#include <cstring>

namespace {
struct Counts {
    long add, mul, div, sqrt, trig;
};
thread_local Counts g_fc;
}  // namespace

struct FlopD {
    double v;
    FlopD() = default;
    FlopD(double x) : v(x) {}  // NOLINT: implicit, as a double literal converts
    explicit operator double() const { return v; }
    FlopD &operator+=(FlopD o) { ++g_fc.add; v += o.v; return *this; }
    FlopD &operator-=(FlopD o) { ++g_fc.add; v -= o.v; return *this; }
    FlopD &operator*=(FlopD o) { ++g_fc.mul; v *= o.v; return *this; }
    FlopD &operator/=(FlopD o) { ++g_fc.div; v /= o.v; return *this; }
};
static_assert(sizeof(FlopD) == sizeof(double), "FlopD must have a double's layout");

inline FlopD operator+(FlopD a, FlopD b) { ++g_fc.add; return FlopD(a.v + b.v); }
inline FlopD operator-(FlopD a, FlopD b) { ++g_fc.add; return FlopD(a.v - b.v); }
inline FlopD operator*(FlopD a, FlopD b) { ++g_fc.mul; return FlopD(a.v * b.v); }
inline FlopD operator/(FlopD a, FlopD b) { ++g_fc.div; return FlopD(a.v / b.v); }
inline FlopD operator-(FlopD a) { return FlopD(-a.v); }
inline bool operator<(FlopD a, FlopD b) { return a.v < b.v; }
inline bool operator<=(FlopD a, FlopD b) { return a.v <= b.v; }
inline bool operator>(FlopD a, FlopD b) { return a.v > b.v; }
inline bool operator>=(FlopD a, FlopD b) { return a.v >= b.v; }
inline bool operator==(FlopD a, FlopD b) { return a.v == b.v; }
inline bool operator!=(FlopD a, FlopD b) { return a.v != b.v; }
inline FlopD sqrt(FlopD a) { ++g_fc.sqrt; return FlopD(std::sqrt(a.v)); }
inline FlopD sin(FlopD a) { ++g_fc.trig; return FlopD(std::sin(a.v)); }
inline FlopD cos(FlopD a) { ++g_fc.trig; return FlopD(std::cos(a.v)); }
inline FlopD acos(FlopD a) { ++g_fc.trig; return FlopD(std::acos(a.v)); }

#define double FlopD
#include "oracle.c"
#undef double

extern "C" {
void oracle_flops_reset(void) { g_fc = Counts{0, 0, 0, 0, 0}; }
// out: add, mul, div, sqrt, trig (sin / cos / acos) since the last reset
void oracle_flops_get(long *out) {
    out[0] = g_fc.add;
    out[1] = g_fc.mul;
    out[2] = g_fc.div;
    out[3] = g_fc.sqrt;
    out[4] = g_fc.trig;
}
}
