"""Operation count of a model-specialised kernel's formulation, per stage (CPU only).

The hipRTC kernels fold the model's constants at compile time: structural zeros drop their
products, +-1 entries their multiplies (jit.cpp).  This tool counts what is left -- the
arithmetic the formulation needs for THIS model once its constants are known -- by compiling the
kernel's own lane bodies (fdh_body / rnea_body / crba_body .hip.hpp, the source
multibody_jit_source_ex emits) for the host with a counting number type `Op`:
  * a value is either a known constant (model data, literals) or a run-time value;
  * x * y, x + y, fma(x, y, z) fold when an operand is a known 0 / +-1 or every operand is known,
    else count one instruction (an FMA counts once; a multiply whose only use is an add is not
    fused here unless the source wrote an fma -- the count is of the source's own operations);
  * negation is free (a source modifier on gfx950);
  * each run-time angle's sincos counts its ISA cost (fp64 table form 15, the fp32 exact
    reduction 4 + 2 transcendental), each reciprocal 3 (v_rcp + one Newton step, 2 FMAs).
Stages follow the RB_STAGE markers the per-stage ISA audit (tools/fd_stages.py) splits on, so
the two tables compare line by line: ISA VALU per stage / op count = how close the compiled code
is to its formulation's minimum.  The input checks (InputGuard) are counted as their own stage.

usage: python tools/opcount.py [fd|rnea|crba] [f64|f32] [DOF] [--json out.json]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rigidbody-rs_amd"))
CSRC = os.path.join(REPO, "rigidbody-rs_amd", "csrc")

PRELUDE = r"""
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <tuple>
static int g_stage = 0;
static std::vector<std::string> g_names = {"loads"};
static std::map<int, long> g_guard;
static void stage(const char *n) {
    for (size_t i = 0; i < g_names.size(); ++i) if (g_names[i] == n) { g_stage = (int)i; return; }
    g_names.push_back(n); g_stage = (int)g_names.size() - 1;
}
#define RB_STAGE(name) stage(name)
// The dataflow graph of the run-time operations (hash-consed: identical operations are one node).
// kind: i input, m mul, a add, f fma, n neg (free), s sincos, p projection (free), r reciprocal.
struct Node { char kind; int a, b, c; int stage; double ka, kb; };
static std::vector<Node> g_nodes;
static std::map<std::tuple<char, int, int, int, double, double>, int> g_hash;
static int node(char kind, int a, int b = -1, int c = -1, double ka = 0, double kb = 0) {
    auto key = std::make_tuple(kind, a, b, c, ka, kb);
    auto it = g_hash.find(key);
    if (it != g_hash.end()) return it->second;
    g_nodes.push_back({kind, a, b, c, g_stage, ka, kb});
    return g_hash[key] = (int)g_nodes.size() - 1;
}
struct Op {
    double v; int id;  // id < 0: a known constant v
    Op() : v(0), id(-1) {}
    Op(double x) : v(x), id(-1) {}
    static Op rt(int id) { Op o; o.id = id; return o; }
    static Op input() { return rt(node('i', (int)g_nodes.size() + 1000000)); }
    bool k() const { return id < 0; }
};
static bool is0(const Op &a) { return a.k() && a.v == 0.0; }
static Op neg(const Op &a) {
    if (a.k()) return Op(-a.v);
    if (g_nodes[a.id].kind == 'n') return Op::rt(g_nodes[a.id].a);  // -(-x) = x
    return Op::rt(node('n', a.id));
}
static bool is_neg(const Op &a) { return !a.k() && g_nodes[a.id].kind == 'n'; }
static Op inner(const Op &a) { return Op::rt(g_nodes[a.id].a); }
static Op operator-(const Op &a) { return neg(a); }
// constant operands are part of the node key (a different constant is a different operation)
static Op operator*(const Op &a, const Op &b) {
    if (a.k() && b.k()) return Op(a.v * b.v);
    // (-x) y = -(x y): one product, the sign a source modifier (as the compiler's CSE sees it)
    if (is_neg(a)) return neg(inner(a) * b);
    if (is_neg(b)) return neg(a * inner(b));
    if (a.k() && a.v < 0 && a.v != -1.0) return neg(Op(-a.v) * b);
    if (b.k() && b.v < 0 && b.v != -1.0) return neg(a * Op(-b.v));
    if (is0(a) || is0(b)) return Op(0.0);
    if (a.k() && a.v == 1.0) return b;
    if (b.k() && b.v == 1.0) return a;
    if (a.k() && a.v == -1.0) return neg(b);
    if (b.k() && b.v == -1.0) return neg(a);
    if (a.k()) return Op::rt(node('m', b.id, -1, -1, a.v));
    if (b.k()) return Op::rt(node('m', a.id, -1, -1, b.v));
    return Op::rt(node('m', a.id < b.id ? a.id : b.id, a.id < b.id ? b.id : a.id));
}
static Op operator+(const Op &a, const Op &b) {
    if (a.k() && b.k()) return Op(a.v + b.v);
    // x + (-x) = 0 (finite math: no NaN / Inf to keep)
    if ((is_neg(b) && !a.k() && inner(b).id == a.id) || (is_neg(a) && !b.k() && inner(a).id == b.id)) return Op(0.0);
    if (is0(a)) return b;
    if (is0(b)) return a;
    if (a.k()) return Op::rt(node('a', b.id, -1, -1, a.v));
    if (b.k()) return Op::rt(node('a', a.id, -1, -1, b.v));
    return Op::rt(node('a', a.id < b.id ? a.id : b.id, a.id < b.id ? b.id : a.id));
}
static Op operator-(const Op &a, const Op &b) { return a + neg(b); }
static Op &operator+=(Op &a, const Op &b) { a = a + b; return a; }
static Op &operator-=(Op &a, const Op &b) { a = a - b; return a; }
static Op &operator*=(Op &a, const Op &b) { a = a * b; return a; }
static Op fmadd(const Op &a, const Op &b, const Op &c) {
    const Op p = a * b;
    if (p.k() || is0(c)) return p + c;
    if (c.k()) return Op::rt(node('f', p.id, -1, -1, c.v));
    return Op::rt(node('f', p.id, c.id));
}
template <bool FAST>
static void sin_cos(const Op &x, Op &s, Op &c) {
    if (x.k()) { s = Op(__builtin_sin(x.v)); c = Op(__builtin_cos(x.v)); return; }
    const int sc = node('s', x.id);
    s = Op::rt(node('p', sc, 0)); c = Op::rt(node('p', sc, 1));
}
static Op recip(const Op &x) { if (x.k()) return Op(1.0 / x.v); return Op::rt(node('r', x.id)); }
static std::vector<int> g_roots;
static void root(const Op &x) { if (!x.k()) g_roots.push_back(x.id); }
// Count the live operations per stage: an 'f' node's product (a mul node) is fused into it when
// the product has no other live use; an add whose one run-time operand is a mul used only there
// fuses likewise (what the compiler's FMA contraction does).
static std::map<int, long> count_live() {
    std::vector<char> live(g_nodes.size(), 0);
    std::vector<int> st(g_roots.begin(), g_roots.end());
    while (!st.empty()) {
        int i = st.back(); st.pop_back();
        if (i < 0 || i >= (int)g_nodes.size() || live[i]) continue;
        live[i] = 1;
        const Node &n = g_nodes[i];
        if (n.kind == 'i') continue;
        for (int o : {n.a, n.b, n.c}) if (o >= 0 && o < (int)g_nodes.size()) st.push_back(o);
    }
    std::vector<int> uses(g_nodes.size(), 0);
    for (size_t i = 0; i < g_nodes.size(); ++i) {
        if (!live[i] || g_nodes[i].kind == 'i') continue;
        for (int o : {g_nodes[i].a, g_nodes[i].b, g_nodes[i].c}) if (o >= 0 && o < (int)g_nodes.size()) uses[o]++;
    }
    auto through_neg = [&](int o) { while (o >= 0 && g_nodes[o].kind == 'n') o = g_nodes[o].a; return o; };
    std::vector<char> fused(g_nodes.size(), 0);
    for (size_t i = 0; i < g_nodes.size(); ++i) {
        if (!live[i]) continue;
        const Node &n = g_nodes[i];
        if (n.kind == 'f' || n.kind == 'a') {
            for (int o : {n.a, n.b}) {
                int m = through_neg(o);
                if (m >= 0 && g_nodes[m].kind == 'm' && uses[m] == 1 && (o == m || uses[o] == 1) && !fused[m]) {
                    fused[m] = 1;
                    break;
                }
            }
        }
    }
    std::map<int, long> per;
    for (size_t i = 0; i < g_nodes.size(); ++i) {
        if (!live[i] || fused[i]) continue;
        const char k = g_nodes[i].kind;
        const long c = k == 'm' || k == 'a' || k == 'f' ? 1 : k == 's' ? SINCOS_OPS : k == 'r' ? 3 : 0;
        per[g_nodes[i].stage] += c;
    }
    return per;
}
"""

GUARD = r"""
namespace rbamd { namespace dev {
// InputGuard on Op: the kernel's checks, counted as their own stage
template <> struct InputGuard<Op> {
    template <int N> void vals(const Op (&x)[N]) { for (int j = 0; j < N; ++j) val(x[j]); }
    template <typename Topo, int N> void joints(const Op (&q)[N]) { for (int j = 0; j < N; ++j) angle(q[j]); }
    void val(const Op &x) { if (!x.k()) g_guard[g_stage] += 1; }
    void angle(const Op &x) { if (!x.k()) g_guard[g_stage] += 2; }
    Op out(const Op &y) const { g_guard[g_stage] += 1; return y; }
};
}}
"""


def build_source(kind, f64, n):
    from rigidbody_amd import chains, ffi

    mb = ffi.Multibody.new() if n == 7 else ffi.Multibody.from_urdf_string(chains.synthetic_chain_urdf(n))
    src = mb.jit_source(f64, kind)
    head, _, _ = src.partition('extern "C" __global__')
    head = head.replace("static __device__ constexpr", "static constexpr")
    # no LDS sincos table on the host: sin_cos is the counting overload above
    head = head.replace("#define RB_SINCOS_TAB 1", "#define RB_SINCOS_TAB 0")
    if "rb_sctab_src" in head:
        a = head.index("static constexpr double rb_sctab_src")
        head = head[:a] + head[head.index("};", a) + 2:]
    # the body headers, with Op in scope, then the guard specialisation
    body_inc = [ln for ln in head.splitlines() if ln.startswith('#include "')]
    rest = "\n".join(ln for ln in head.splitlines() if not ln.startswith('#include "'))
    sincos = 15 if f64 else 6
    main = {
        "fd": r"""
int main() {
    using namespace rbamd::dev;
    Op m[sizeof(kModel) / sizeof(kModel[0])];
    for (size_t i = 0; i < sizeof(kModel) / sizeof(kModel[0]); ++i) m[i] = Op((double)kModel[i]);
    Op q[N], qd[N];
    for (int j = 0; j < N; ++j) { q[j] = Op::input(); qd[j] = Op::input(); }
    fdh_eval<Op, N, true>(m, q, qd, [&](Op (&tv)[N]) { for (int j = 0; j < N; ++j) tv[j] = Op::input(); },
                          [&](int, Op v) { root(v); });
    report();
}""",
        "rnea": r"""
int main() {
    using namespace rbamd::dev;
    Op m[sizeof(kModel) / sizeof(kModel[0])];
    for (size_t i = 0; i < sizeof(kModel) / sizeof(kModel[0]); ++i) m[i] = Op((double)kModel[i]);
    Op q[N], qd[N], qdd[N];
    for (int j = 0; j < N; ++j) { q[j] = Op::input(); qd[j] = Op::input(); qdd[j] = Op::input(); }
    stage("fwd");
    rnea_eval<Op, N, true>(m, q, qd, qdd, [&](int, Op v) { root(v); });
    report();
}""",
        "crba": r"""
int main() {
    using namespace rbamd::dev;
    Op m[sizeof(kModel) / sizeof(kModel[0])];
    for (size_t i = 0; i < sizeof(kModel) / sizeof(kModel[0]); ++i) m[i] = Op((double)kModel[i]);
    Op q[N];
    for (int j = 0; j < N; ++j) q[j] = Op::input();
    stage("crba");
    crba_eval<Op, N, true>(m, q, [&](int, Op v) { root(v); });
    report();
}""",
    }[kind]
    report = r"""
static void report() {
    long tot = 0, gtot = 0;
    std::map<int, long> g_ops = count_live();
    printf("{\"stages\": [");
    for (size_t i = 0; i < g_names.size(); ++i) {
        tot += g_ops[(int)i]; gtot += g_guard[(int)i];
        printf("%s{\"stage\": \"%s\", \"ops\": %ld, \"guard_ops\": %ld}", i ? ", " : "", g_names[i].c_str(),
               g_ops[(int)i], g_guard[(int)i]);
    }
    printf("], \"ops_total\": %ld, \"guard_total\": %ld}\n", tot, gtot);
}
"""
    text = ("#define SINCOS_OPS %d\n" % sincos + "#include <hip/hip_runtime.h>\n" + PRELUDE
            + "\n".join(body_inc) + "\n" + GUARD + rest.replace("using T = double;", "").replace("using T = float;", "")
            + report + main)
    # the kernel's model array is typed T; keep it double on the host
    text = text.replace("static constexpr T kModel", "static constexpr double kModel")
    return text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", nargs="?", default="fd", choices=["fd", "rnea", "crba"])
    ap.add_argument("dt", nargs="?", default="f64", choices=["f64", "f32"])
    ap.add_argument("dof", nargs="?", type=int, default=7)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    text = build_source(a.kind, a.dt == "f64", a.dof)
    d = tempfile.mkdtemp(prefix="opcount_")
    cpp = os.path.join(d, "oc.hip")
    open(cpp, "w").write(text)
    exe = os.path.join(d, "oc")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--cuda-host-only", "-O1", "-std=c++17", "-I", CSRC,
                        "-Wno-unused-function", "-Wno-unused-variable", "-o", exe, cpp],
                       capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-6000:] + f"\n(source: {cpp})")
    out = json.loads(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)
    out.update({"kind": a.kind, "dtype": a.dt, "dof": a.dof})
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
