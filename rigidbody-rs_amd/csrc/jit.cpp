// jit.cpp -- see jit.hpp.
#include "jit.hpp"

#include <hip/hiprtc.h>

#include <algorithm>
#include <string_view>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <vector>

#include "jit_sources.inc"  // kJitHeaderNames / kJitHeaderSources (tools/embed_sources.py)
#include "layout.hpp"
#include "tuning.hpp"

namespace rbamd {

bool jit_enabled() { return tuning().jit != 0; }

namespace {

double snap(double x) {
    if (std::fabs(x) < 1e-14) return 0.0;
    if (std::fabs(x - 1.0) < 1e-14) return 1.0;
    if (std::fabs(x + 1.0) < 1e-14) return -1.0;
    return x;
}

std::string literal(double x, bool f64) {
    char buf[64];
    if (x == 0.0) return f64 ? "0.0" : "0.0f";
    if (f64)
        std::snprintf(buf, sizeof buf, "%.17g", x);
    else
        std::snprintf(buf, sizeof buf, "%.9gf", (double)(float)x);
    std::string s(buf);
    // make sure an integral value still reads as a floating literal
    if (s.find_first_of(".eEn") == std::string::npos) s.insert(f64 ? s.size() : s.size() - 1, ".0");
    return s;
}

}  // namespace

int jit_nt(JitKind kind) {
    if (kind == JitKind::Rnea) return tuning().rnea_nt < 0 ? 3 : (tuning().rnea_nt & 3);
    if (kind == JitKind::Fd || kind == JitKind::Rollout || kind == JitKind::RneaFd) return tuning().fd_nt & 3;
    const int v = tuning().kin_nt;  // CRBA, fwd_kin, jac
    if (v >= 0) return v & 3;
    return kind == JitKind::FwdKin ? 3 : 2;  // 7 rows in / 3 out: non-temporal loads pay too
}

// Rollouts whose K loop must not hoist anything (machine LICM off, the row stride re-derived
// per step): the paired fp32 form, and fp64 chains up to 8 links -- 212 instead of 264 VGPRs,
// 2 waves/SIMD instead of 1: FR3 2^20 x 16 steps 641 vs 1027 us (12 links: no change; 30
// links, state in registers: 6.09 vs 5.81 ms, so not there).
bool jit_rollout_no_hoist(bool f64, int n, int pack) { return pack == 2 || pack == 4 || (f64 && n <= 8); }

bool jit_opaque(JitKind kind, bool f64, int n) {
    const int v = tuning().opaque_consts;
    if (v >= 0) return v != 0;
    // fp64 short-chain rollouts: with hoisting off, SGPR-pinned fp64 constants only spill
    return n <= 16 && kind == JitKind::Rollout && !(f64 && n <= 8);
}

int jit_waves(JitKind kind, bool f64, int n) {
    const int v = tuning().jit_waves;
    if (v >= 0) return v;
    if (kind == JitKind::Rollout && !f64 && n <= 8) return jit_pack(kind, f64, n) != 1 ? 2 : 4;
    // (the fp64 rollout of the mass-matrix form takes a 4-wave target in jit_source; the ABA
    // form -- the rollout of trees, or fd_form 1 -- none: 436 B of scratch per lane under it)
    return 0;
}

int jit_pack(JitKind kind, bool f64, int n) {
    // 2 = two configurations per lane on packed fp32 (fp32 forward dynamics of chains up to 8
    // links: FR3 2^20 tiled 28.7 vs 30.7 us; 200+ VGPRs for the pair, 2 waves/SIMD; the
    // 30-link chain needs ~240 VGPRs for one configuration).  The RNEA pair (128 VGPRs, 4
    // waves/SIMD instead of 8) measured slower, 22.6 vs 21.0 us, and was removed.  The fp32
    // rollout of chains up to 8 links is paired too (rollout_lane2: 251 VGPRs, 2 waves/SIMD,
    // constants pinned in SGPRs and machine LICM off so the K loop hoists nothing; FR3 2^20
    // x 16 steps 317-323 vs 333-335 us one per lane at 4 waves/SIMD).
    // 3 = two configurations per lane evaluated one after the other from one load burst (the
    // fp64 RNEA of chains up to 8 links: 125 VGPRs, still 4 waves/SIMD; FR3 2^20 tiled
    // 42.0-42.8 us steady where the one-per-lane kernel alternates between ~40.7 and ~48.8 us
    // phases, mean 44.3-44.6).
    const int v = tuning().pack;
    if (kind == JitKind::Rollout) return ((v < 0 || v == 2 || v == 4) && !f64 && n <= 8) ? (v == 4 ? 4 : 2) : 1;
    // the fused inverse + forward dynamics: one per lane, or its wave split (idfd_split_block1)
    if (kind == JitKind::RneaFd) return v == 5 ? 5 : 1;
    if (kind != JitKind::Fd && kind != JitKind::Rnea) return 1;
    if (v == 3) return 3;
    if (v == 4) return (kind == JitKind::Fd && !f64) ? 4 : 1;  // split packed waves (fdh_split_block2)
    if (v == 5) return kind == JitKind::Fd ? 5 : 1;             // split waves, one per lane (fdh_split_block1)
    if (v >= 0) return (v >= 2 && !f64 && kind == JitKind::Fd) ? 2 : 1;
    if (kind == JitKind::Rnea) return (f64 && n <= 8) ? 3 : 1;
    return (!f64 && n <= 8) ? 2 : 1;
}

bool jit_f64_tab(bool f64) { return f64 && tuning().f64_tab != 0; }

int jit_fd_form(const Model &m, JitKind kind) {
    // 2 = mass-matrix forward dynamics (fdh_body.hip.hpp: RNEA bias + CRBA + L D L^T), 1 = the
    // Articulated-Body Algorithm (aba_body.hip.hpp).  The mass-matrix form holds ~n^2/2 values
    // per lane where the ABA holds ~12 per link across its sweeps, so it runs at 2-3x the
    // ABA's waves per SIMD on short chains; its O(n^2) work loses on long ones.  Trees keep
    // the ABA (tree_body.hip.hpp).  Forward dynamics: the mass-matrix form up to 12 links (12
    // links 2^20 tiled: fp64 119.0 vs 159.5 us on the ABA -- 242 registers, 2 waves/SIMD, against
    // the ABA's 398, 1 wave -- fp32 64.6 vs 75.6; 16 links: the ABA, 224 vs 229 / 101 vs 113;
    // profiles/r05/ab/fd_form/).  Rollouts: up to 8 links (12 links x 16 steps: the ABA 2205 vs
    // 3141 us fp64, 920 vs 959 fp32).
    const int v = tuning().fd_form;
    // trees: the mass-matrix form only for forward dynamics and only on request (fdh_eval_tree;
    // A/B), rollouts and the wave splits / pairs are serial-chain forms
    if (!m.serial_revolute()) return (kind == JitKind::Fd && v == 2) ? 2 : 1;
    if (v == 1 || v == 2) return v;
    return m.n <= (kind == JitKind::Rollout ? 8 : 12) ? 2 : 1;
}

int jit_seq_tail(bool tiled) {
    const int v = tuning().seq_tail;
    if (v < 0) return tiled ? 75 : 0;
    return v < 100 ? v : 100;
}

int jit_model_pack(const Model &m, JitKind kind, bool f64, int pack_req) {
    const int pack = pack_req > 0 ? pack_req : jit_pack(kind, f64, m.n);
    // the tree form of the mass-matrix forward dynamics is one configuration per lane
    if (kind == JitKind::Fd && !m.serial_revolute() && jit_fd_form(m) == 2) return 1;
    // the mass-matrix forward dynamics has one- and two-per-lane forms only
    if (kind == JitKind::Fd && pack == 3 && jit_fd_form(m) == 2) return 1;
    // 4 / 5 = the bias / mass-matrix wave split, packed / one per lane: fp32 mass-matrix FD only
    if (pack == 4 && kind == JitKind::Rollout && !(!f64 && jit_fd_form(m, kind) == 2 && !(tuning().jit_variant & 256)))
        return (!f64 && m.n <= 8) ? 2 : 1;  // the split needs the mass-matrix form: the pair instead
    if (pack == 4 && kind != JitKind::Rollout && !(kind == JitKind::Fd && !f64 && jit_fd_form(m) == 2)) return 1;
    if (pack == 5 && !((kind == JitKind::Fd || kind == JitKind::RneaFd) && jit_fd_form(m) == 2 && m.serial_revolute()))
        return 1;
    return pack;
}

std::string jit_tag(JitKind kind, bool f64, int n) {
    // ":w" the policy's target, ":W" the raw knob (-1 lets jit_compile rebuild at the occupancy cliff)
    return ":nt" + std::to_string(jit_nt(kind)) + ":w" + std::to_string(jit_waves(kind, f64, n)) + ":W" +
           std::to_string(tuning().jit_waves.load()) + ":o" +
           std::to_string(jit_opaque(kind, f64, n) ? 1 : 0) + ":p" + std::to_string(jit_pack(kind, f64, n)) +
           ":t" + std::to_string(jit_f64_tab(f64) ? 1 : 0) + ":r" + std::to_string(tuning().split_rot) + ":v" +
           std::to_string(tuning().jit_variant) + ":f" + std::to_string(tuning().fd_form) + ":k" +
           std::to_string(kind == JitKind::Rnea ? tuning().rnea_park.load() : 0) + ":e" +
           std::to_string(kind == JitKind::Rnea ? tuning().rnea_rev.load() : 0) + ":a" +
           std::to_string(tuning().kernarg_preload.load());
}

int code_vgprs(const std::vector<char> &code) {
    // msgpack map entry ".vgpr_count" (fixstr 0xab) -> positive fixint / uint8 (0xcc) / uint16 (0xcd)
    static const char key[] = "\xab.vgpr_count";
    const std::string_view buf(code.data(), code.size());
    const size_t at = buf.find(std::string_view(key, sizeof(key) - 1));
    if (at == std::string_view::npos) return -1;
    size_t i = at + sizeof(key) - 1;
    if (i >= buf.size()) return -1;
    const unsigned char t = (unsigned char)buf[i];
    if (t < 0x80) return t;
    if (t == 0xcc && i + 1 < buf.size()) return (unsigned char)buf[i + 1];
    if (t == 0xcd && i + 2 < buf.size()) return ((unsigned char)buf[i + 1] << 8) | (unsigned char)buf[i + 2];
    return -1;
}

std::string jit_source(const Model &m, JitKind kind, bool f64, bool fast, int pack_req, int tail, int nt,
                       int waves_req) {
    std::vector<double> pk = m.pack_f64();
    for (int i = 0; i < m.n; ++i) {
        double *c = &pk[(size_t)i * kLinkStride];
        for (int k = 0; k < 9; ++k) c[kE0 + k] = snap(c[kE0 + k]);
        for (int k = 0; k < 3; ++k) c[kP + k] = snap(c[kP + k]);
    }
    const char *F = fast ? "true" : "false";
    const int pack = jit_model_pack(m, kind, f64, pack_req);
    const bool fdh = (kind == JitKind::Fd || kind == JitKind::RneaFd) && jit_fd_form(m) == 2;
    std::ostringstream o;
    o << "#define RB_NT " << (nt >= 0 ? nt : jit_nt(kind)) << "\n";
    o << "#define RB_VARIANT " << tuning().jit_variant << "\n";
    o << "#define RB_OPAQUE_CONSTS " << (jit_opaque(kind, f64, m.n) ? 1 : 0) << "\n";
    if (kind == JitKind::Rollout && jit_rollout_no_hoist(f64, m.n, pack)) o << "#define RB_ROLLOUT_NO_HOIST 1\n";
    // input checks pinned into the sweep's state (rnea_body.hip.hpp rnea_fwd)
    if (kind == JitKind::Rollout || m.n > 8) o << "#define RB_GUARD_ANCHOR 1\n";
    // the rollout's forward dynamics follows the fd_form policy (mass-matrix form for short
    // serial chains) unless RB_VARIANT bit 8 (A/B) keeps the ABA
    if (kind == JitKind::Rollout && jit_fd_form(m, kind) == 2 && !(tuning().jit_variant & 256))
        o << "#define RB_ROLLOUT_FDH 1\n";
    const bool tab = jit_f64_tab(f64);
    o << "#define RB_SINCOS_TAB " << (tab ? 1 : 0) << "\n";
    if (tab) {  // (cos, sin)(k pi/128), k < 256, for sincos_tab (spatial.hip.hpp): long double, quadrants exact
        const long double pi = 3.141592653589793238462643383279502884L;
        o << "static __device__ constexpr double rb_sctab_src[512] = {\n";
        for (int k = 0; k < 256; ++k) {
            double c = (double)std::cos((long double)k * pi / 128.0L), s = (double)std::sin((long double)k * pi / 128.0L);
            if (k % 64 == 0) {
                const int q = k / 64;
                c = q == 0 ? 1.0 : q == 2 ? -1.0 : 0.0;
                s = q == 1 ? 1.0 : q == 3 ? -1.0 : 0.0;
            }
            o << "  " << literal(c, true) << ", " << literal(s, true) << ",\n";
        }
        o << "};\n";
    }
    // Split joint rotation (artinertia.hip.hpp to_parent_split): pays only when every R_p is a
    // signed permutation (its congruence then folds away); a dense constant R_p (general-axis
    // frames, trees) makes it costlier than the folded E S E^T.
    bool perm = true;
    for (int i = 0; i < m.n && perm; ++i)
        for (int r = 0; r < 3; ++r) {
            int ones = 0;
            for (int c = 0; c < 3; ++c) {
                const double v = pk[(size_t)i * kLinkStride + kE0 + 3 * r + c];
                if (v == 1.0 || v == -1.0) ++ones;
                else if (v != 0.0) perm = false;
            }
            if (ones != 1) perm = false;
        }
    const int sr = tuning().split_rot;
    o << "#define RB_SPLIT_ROT " << ((sr > 0 || (sr < 0 && perm)) ? 1 : 0) << "\n";
    // Newton-Euler link forces about the centre of mass (spatial.hip.hpp link_force) for the
    // RNEA sweeps of chains and trees (and so the mass-matrix FD's bias): c = h / m and
    // Ic = I_o - m (|c|^2 1 - c c^T) per link (massless virtual links: c = 0, Ic = I_o = 0), in
    // fp64 here.  jit_variant bit 9 (A/B) keeps the origin form.  Not for the fp64 RNEA of chains
    // up to 8 links (the reversed long-chain form below takes it): the
    // memory-bound headline kernel gains nothing from fewer VALU, its sequential pair would need
    // 131 instead of 125 VGPRs (3 waves/SIMD instead of 4), and all its grid forms (pairs,
    // single tail, one per lane below 2^19) must stay bit-identical to each other.
    const bool dyn = kind == JitKind::Rnea || kind == JitKind::Fd || kind == JitKind::Rollout || kind == JitKind::RneaFd;
    // jit_variant bit 16384 (A/B): the centre-of-mass form for the fp64 RNEA too
    // rnea_lane_rev: the fp64 RNEA of serial chains longer than 8 links, whose per-link forces
    // hold one wave per SIMD (12 links 264 VGPRs, 30 links 496) and do not fit LDS either
    // (rnea_park's fp64 forces would take 60 KB per wave); centre-of-mass link forces, any joint
    // frames (general axes included)
    const bool rev = kind == JitKind::Rnea && f64 && m.n > 8 && m.serial_revolute() && tuning().rnea_rev != 0;
    const bool com = dyn && !(kind == JitKind::Rnea && f64 && !rev && !(tuning().jit_variant & 16384)) &&
                     !(tuning().jit_variant & 512);
    // rnea_lane_park: fp32 one-per-lane RNEA of long serial chains in the centre-of-mass g-form
    // (signed-permutation frames), when the tuning asks for it
    // the parked forces take NP x 6 KB of LDS per 4-wave block: at most kMaxPark links, so that 3
    // blocks still fit a CU's 160 KB (gfx950) -- a requested count past it is clamped, not handed to
    // hipRTC to fail on (which would leave the launch on the generic kernel)
    constexpr int kMaxPark = (160 * 1024 / 3) / (4 * 6 * 64 * 4);
    const int pk_req = std::min(kMaxPark, tuning().rnea_park < 0 ? (m.n >= 20 ? 8 : 0) : tuning().rnea_park.load());
    const int park = (kind == JitKind::Rnea && !f64 && pack == 1 && m.serial_revolute() && com &&
                      (sr > 0 || (sr < 0 && perm)) && pk_req > 0 && pk_req < m.n) ? pk_req : 0;
    if (com) {
        o << "#define RB_COM_FORM 1\n";
        o << "static __device__ constexpr double rb_com[" << 9 * m.n << "] = {\n";
        for (int i = 0; i < m.n; ++i) {
            const double *L = &pk[(size_t)i * kLinkStride];
            const double mass = L[kM];
            double c[3] = {0, 0, 0};
            if (mass > 0)
                for (int k = 0; k < 3; ++k) c[k] = L[kH + k] / mass;
            const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
            const double Ic[6] = {L[kIo + 0] - mass * (cc - c[0] * c[0]), L[kIo + 1] + mass * c[0] * c[1],
                                  L[kIo + 2] + mass * c[0] * c[2],        L[kIo + 3] - mass * (cc - c[1] * c[1]),
                                  L[kIo + 4] + mass * c[1] * c[2],        L[kIo + 5] - mass * (cc - c[2] * c[2])};
            o << "  ";
            for (int k = 0; k < 3; ++k) o << literal(c[k], true) << ", ";
            for (int k = 0; k < 6; ++k) o << literal(Ic[k], true) << ", ";
            o << "\n";
        }
        o << "};\n";
    }
    o << (kind == JitKind::Rnea                               ? "#include \"rnea_body.hip.hpp\"\n"
          : fdh                                               ? "#include \"fdh_body.hip.hpp\"\n"
          : (kind == JitKind::Fd || kind == JitKind::Rollout) ? "#include \"aba_body.hip.hpp\"\n"
          : kind == JitKind::Crba                             ? "#include \"crba_body.hip.hpp\"\n"
                                                              : "#include \"tree_body.hip.hpp\"\n");
    o << "using T = " << (f64 ? "double" : "float") << ";\n";
    o << "constexpr int N = " << m.n << ";\n";
    // Topology policy (tree_body.hip.hpp): the tuned serial code for the reference's chain,
    // else the tree forms with every parent index / joint type a compile-time constant.
    if (m.serial_revolute()) {
        o << "using Topo = rbamd::dev::SerialTopo;\n";
    } else {
        o << "struct Topo {\n  static constexpr bool kSerial = false;\n  static constexpr int kPar[N] = {";
        for (int i = 0; i < m.n; ++i) o << (i ? ", " : "") << m.links[i].parent;
        o << "};\n  static constexpr int kPri[N] = {";
        for (int i = 0; i < m.n; ++i) o << (i ? ", " : "") << (m.links[i].type == kJointPrismatic ? 1 : 0);
        o << "};\n"
             "  static constexpr int parent(int j) { return kPar[j]; }\n"
             "  static constexpr bool prismatic(int j) { return kPri[j] != 0; }\n"
             "  static constexpr int last_child(int j) { int c = -1; for (int k = j + 1; k < N; ++k) if (kPar[k] == j) c = k; return c; }\n"
             "  static constexpr bool is_ancestor(int a, int i) { for (int k = kPar[i]; k >= 0; k = kPar[k]) if (k == a) return true; return false; }\n"
             "  static constexpr int child_toward(int a, int i) { int c = i; for (int k = kPar[i]; k >= 0; c = k, k = kPar[k]) if (k == a) return c; return -1; }\n"
             "  static constexpr bool on_path(int j) { return j == N - 1 || is_ancestor(j, N - 1); }\n"
             "};\n";
    }
    if (pack == 2 || pack == 4) {  // paired fp32 lanes: every constant splat to both halves (spatial.hip.hpp f2)
        o << "using TV = rbamd::dev::f2;\n";
        o << "static __device__ constexpr TV kModel[" << pk.size() << "] = {\n";
        for (size_t k = 0; k < pk.size(); ++k) {
            const std::string c = literal(pk[k], f64);
            o << "  TV{" << c << ", " << c << "},\n";
        }
    } else {
        o << "static __device__ constexpr T kModel[" << pk.size() << "] = {\n";
        for (size_t k = 0; k < pk.size(); ++k) o << "  " << literal(pk[k], f64) << ",\n";
    }
    o << "};\n";
    // Paired lanes: block k owns batch blocks 2k and 2k+1 (SoA: configurations 512k + t and
    // 512k + 256 + t; tiled: lane t of tiles 2k and 2k+1).  When the second is past B, the
    // lane evaluates the first twice and stores the bit-identical value twice.
    const char *pair_prologue =
        "  const uint32_t bA = blockIdx.x * 512u + threadIdx.x;\n"
        "  if (bA >= B) return;\n"
        "  const int64_t oA = (int64_t)(2u * blockIdx.x) * bs;\n"
        "  const uint32_t offA = threadIdx.x * 4u;\n"
        "  const uint32_t offB = bA + 256u < B ? offA + (uint32_t)bs * 4u : offA;\n";
    // Sequential pair (pack 3): lane t of batch blocks 2k and 2k+1, evaluated one after the
    // other from one load burst; the second only when it exists (twoB).
    const std::string seq_prologue =
        "  const uint32_t bA = blockIdx.x * 512u + threadIdx.x;\n"
        "  if (bA >= B) return;\n"
        "  const int64_t oA = (int64_t)(2u * blockIdx.x) * bs;\n"
        "  const uint32_t offA = threadIdx.x * (uint32_t)sizeof(T);\n"
        "  const bool twoB = bA + 256u < B;\n"
        "  const uint32_t offB = offA + (uint32_t)bs * (uint32_t)sizeof(T);\n";
    std::string head_s = "extern \"C\" __global__ __launch_bounds__(256) ";
    // The paired mass-matrix FD fits 4 waves/SIMD at exactly 128 VGPRs with the occupancy
    // target (130 and 3 waves without): FR3 2^20 tiled 26.4 vs 27.0 us.
    int waves = waves_req >= 0 ? waves_req : jit_waves(kind, f64, m.n);
    if (fdh && pack == 2 && tuning().jit_waves < 0 && waves_req < 0) waves = 4;
    // fp64 rollout of the mass-matrix form: 127 VGPRs, 4 waves/SIMD either way since the input
    // checks; the target keeps it there (FR3 2^20 x 16 steps, reset state: 690-708 vs 702-704 us,
    // noise-level).  Not for the ABA form: 256 VGPRs at 1 wave/SIMD runs 984 us, 2 / 3 / 4-wave
    // targets spill (1068 / 2756 / 4131 us; profiles/r05/ab/rollout_forms/).
    if (kind == JitKind::Rollout && f64 && m.n <= 8 && jit_fd_form(m, kind) == 2 && !(tuning().jit_variant & 256) &&
        tuning().jit_waves < 0 && waves_req < 0)
        waves = 4;
    if (kind == JitKind::Rnea && f64 && (tuning().jit_variant & 32768) && tuning().jit_waves < 0 && waves_req < 0)
        waves = 4;  // A/B
    if (const int w = waves)
        head_s += "__attribute__((amdgpu_waves_per_eu(" + std::to_string(w) + "))) ";
    head_s += "void ";
    const char *head = head_s.c_str();
    // Lane kernels take the block stride bs (elements): 256 for SoA, N * 256 for the tiled
    // layout (kernels.hpp); block k's arrays start at element k * bs, lane offset threadIdx.x.
    if (kind == JitKind::Rnea && pack == 3 && tail > 0) {
        // pairs of tiles for blocks < G1, then one tile per block for the last S tiles
        o << head << "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ qdd, T *__restrict__ tau, uint32_t B, int64_t ld, int64_t bs) {\n";
        o << "  const uint32_t T_ = (B + 255u) / 256u, S_ = (uint32_t)(((uint64_t)T_ * " << tail
          << "u) / 100u);\n";
        o << "  const uint32_t P_ = (T_ - S_) & ~1u, G1 = P_ / 2u;\n";
        o << "  if (blockIdx.x >= G1) {\n";
        o << "    const uint32_t t = P_ + (blockIdx.x - G1), b = t * 256u + threadIdx.x;\n";
        o << "    if (b >= B) return;\n";
        o << "    const int64_t o = (int64_t)t * bs;\n";
        o << "    rbamd::dev::rnea_lane<T, N, " << F
          << ", Topo>(kModel, q + o, qd + o, qdd + o, tau + o, threadIdx.x, ld);\n    return;\n  }\n";
        o << seq_prologue;
        o << "  rbamd::dev::rnea_lane_seq2<T, N, " << F
          << ", Topo>(kModel, q + oA, qd + oA, qdd + oA, tau + oA, offA, offB, twoB, ld);\n}\n";
    } else if (kind == JitKind::Rnea && pack == 3) {
        o << head << "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ qdd, T *__restrict__ tau, uint32_t B, int64_t ld, int64_t bs) {\n";
        o << seq_prologue;
        o << "  rbamd::dev::rnea_lane_seq2<T, N, " << F
          << ", Topo>(kModel, q + oA, qd + oA, qdd + oA, tau + oA, offA, offB, twoB, ld);\n}\n";
    } else if (kind == JitKind::Rnea && rev && com && pack == 1) {
        o << head << "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ qdd, T *__restrict__ tau, uint32_t B, int64_t ld, int64_t bs) {\n";
        o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
        o << "  if (b >= B) return;\n";
        o << "  const int64_t o = (int64_t)blockIdx.x * bs;\n";
        o << "  rbamd::dev::rnea_lane_rev<T, N, " << F << ">(kModel, q + o, qd + o, qdd + o, tau + o, threadIdx.x, ld);\n}\n";
    } else if (kind == JitKind::Rnea && park > 0) {
        o << "extern \"C\" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void "
             "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ qdd, T *__restrict__ tau, uint32_t B, int64_t ld, int64_t bs) {\n";
        o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
        o << "  if (b >= B) return;\n";
        o << "  const int64_t o = (int64_t)blockIdx.x * bs;\n";
        o << "  rbamd::dev::rnea_lane_park<T, N, " << F << ", " << park
          << ">(kModel, q + o, qd + o, qdd + o, tau + o, threadIdx.x, ld);\n}\n";
    } else if (kind == JitKind::Rnea) {
        o << head << "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ qdd, T *__restrict__ tau, uint32_t B, int64_t ld, int64_t bs) {\n";
        o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
        o << "  if (b >= B) return;\n";
        o << "  const int64_t o = (int64_t)blockIdx.x * bs;\n";
        o << "  rbamd::dev::rnea_lane<T, N, " << F << ", Topo>(kModel, q + o, qd + o, qdd + o, tau + o, threadIdx.x, ld);\n}\n";
    } else if (kind == JitKind::RneaFd) {
        // one configuration per lane; the launcher takes this kind only for mass-matrix models
        o << head << "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ qdd, const T *__restrict__ tau_in, T *__restrict__ tau, "
             "T *__restrict__ qdd_out, uint32_t B, int64_t ld, int64_t bs) {\n";
        if (pack == 5) {
            o << "  rbamd::dev::idfd_split_block1<T, N, " << F << ">(kModel, q, qd, qdd, tau_in, tau, qdd_out, B, ld, bs);\n}\n";
        } else {
            o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
            o << "  if (b >= B) return;\n";
            o << "  const int64_t o = (int64_t)blockIdx.x * bs;\n";
            o << "  rbamd::dev::idfd_lane<T, N, " << F
              << ">(kModel, q + o, qd + o, qdd + o, tau_in + o, tau + o, qdd_out + o, threadIdx.x, ld);\n}\n";
        }
    } else if (kind == JitKind::Fd) {
        o << head << "rb_jit_kernel(const T *__restrict__ q, const T *__restrict__ qd, "
             "const T *__restrict__ tau, T *__restrict__ qdd, uint32_t B, int64_t ld, int64_t bs) {\n";
        if (fdh && pack == 5) {
            o << "  rbamd::dev::fdh_split_block1<T, N, " << F << ">(kModel, q, qd, tau, qdd, B, ld, bs);\n}\n";
        } else if (fdh && pack == 4) {
            o << "  rbamd::dev::fdh_split_block2<N, " << F << ">(kModel, q, qd, tau, qdd, B, ld, bs);\n}\n";
        } else if (fdh && pack == 2) {
            o << pair_prologue;
            o << "  rbamd::dev::fdh_lane2<N, " << F << ">(kModel, q + oA, qd + oA, tau + oA, qdd + oA, offA, offB, ld);\n}\n";
        } else if (fdh) {
            o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
            o << "  if (b >= B) return;\n";
            o << "  const int64_t o = (int64_t)blockIdx.x * bs;\n";
            o << "  rbamd::dev::fdh_lane<T, N, " << F << ", Topo>(kModel, q + o, qd + o, tau + o, qdd + o, threadIdx.x, ld);\n}\n";
        } else if (pack == 3) {
            o << seq_prologue;
            o << "  rbamd::dev::aba_lane_seq2<T, N, " << F
              << ", Topo>(kModel, q + oA, qd + oA, tau + oA, qdd + oA, offA, offB, twoB, ld);\n}\n";
        } else if (pack == 2) {
            o << pair_prologue;
            o << "  rbamd::dev::aba_lane2<N, " << F
              << ", Topo>(kModel, q + oA, qd + oA, tau + oA, qdd + oA, offA, offB, ld);\n}\n";
        } else {
            o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
            o << "  if (b >= B) return;\n";
            o << "  const int64_t o = (int64_t)blockIdx.x * bs;\n";
            o << "  rbamd::dev::aba_lane<T, N, " << F << ", Topo>(kModel, q + o, qd + o, tau + o, qdd + o, threadIdx.x, ld);\n}\n";
        }
    } else if (kind == JitKind::Rollout && pack == 4) {
        o << head << "rb_jit_kernel(T *__restrict__ q, T *__restrict__ qd, const T *__restrict__ tau_seq, T dt, "
             "int K, T *__restrict__ traj, uint32_t B, int64_t ld) {\n";
        o << "  rbamd::dev::rollout_split_block2<N, " << F << ">(kModel, q, qd, tau_seq, dt, K, traj, B, ld);\n}\n";
    } else if (kind == JitKind::Rollout && pack == 2) {
        o << head << "rb_jit_kernel(T *__restrict__ q, T *__restrict__ qd, const T *__restrict__ tau_seq, T dt, "
             "int K, T *__restrict__ traj, uint32_t B, int64_t ld) {\n";
        o << "  __shared__ rbamd::dev::RolloutShared2<N> sh;\n";
        o << "  const uint32_t bA = blockIdx.x * 512u + threadIdx.x;\n";
        o << "  if (bA >= B) return;\n";
        o << "  const uint32_t offA = bA * 4u, offB = bA + 256u < B ? offA + 1024u : offA;\n";
        o << "  rbamd::dev::rollout_lane2<N, " << F << ", Topo>(kModel, q, qd, tau_seq, dt, K, traj, offA, offB, ld, sh);\n}\n";
    } else if (kind == JitKind::Rollout) {
        o << head << "rb_jit_kernel(T *__restrict__ q, T *__restrict__ qd, const T *__restrict__ tau_seq, T dt, "
             "int K, T *__restrict__ traj, uint32_t B, int64_t ld) {\n";
        o << "  __shared__ rbamd::dev::RolloutShared<T, N> sh;\n";
        o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
        o << "  if (b >= B) return;\n";
        o << "  rbamd::dev::rollout_lane<T, N, " << F << ", Topo>(kModel, q, qd, tau_seq, dt, K, traj, b, ld, sh);\n}\n";
    } else if (kind == JitKind::FwdKin || kind == JitKind::Jac) {
        // q-only kernels take the block strides of their input and output rows (256 for SoA;
        // n * 256 / rows * 256 for the tiled layout), as the lane kernels above
        o << head << "rb_jit_kernel(const T *__restrict__ q, T *__restrict__ out, uint32_t B, int64_t ld, "
             "int64_t bs_in, int64_t bs_out) {\n";
        o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
        o << "  if (b >= B) return;\n";
        o << "  rbamd::dev::" << (kind == JitKind::FwdKin ? "fwd_kin" : "jac") << "_lane_tree<T, N, " << F
          << ", Topo>(kModel, q + (int64_t)blockIdx.x * bs_in, out + (int64_t)blockIdx.x * bs_out, threadIdx.x, ld);\n}\n";
    } else {
        o << head << "rb_jit_kernel(const T *__restrict__ q, T *__restrict__ H, uint32_t B, int64_t ld, "
             "int64_t bs_in, int64_t bs_out) {\n";
        o << "  const uint32_t b = blockIdx.x * 256u + threadIdx.x;\n";
        o << "  if (b >= B) return;\n";
        o << "  rbamd::dev::crba_lane<T, N, " << F
          << ", Topo>(kModel, q + (int64_t)blockIdx.x * bs_in, H + (int64_t)blockIdx.x * bs_out, threadIdx.x, ld);\n}\n";
    }
    std::string src = o.str();
    if (tab) {  // every kernel fills the block's sincos table first (all lanes still present)
        const size_t at = src.find("rb_jit_kernel(");
        const size_t body = at == std::string::npos ? at : src.find(") {\n", at);
        if (body != std::string::npos) src.insert(body + 4, "  rbamd::dev::sctab_init();\n");
    }
    return src;
}

namespace {
bool rtc_compile(const std::string &src, const std::string &arch, bool no_licm, std::vector<char> *code,
                 std::string *error) {
    hiprtcProgram prog = nullptr;
    if (hiprtcCreateProgram(&prog, src.c_str(), "rb_jit.hip", kJitHeaderCount, kJitHeaderSources,
                            kJitHeaderNames) != HIPRTC_SUCCESS) {
        *error = "hiprtcCreateProgram failed";
        return false;
    }
    const std::string arch_opt = "--offload-arch=" + arch;
    const char *opts[] = {arch_opt.c_str(), "-O3", "-std=c++17", "-ffinite-math-only", "-fno-signed-zeros"};
    std::vector<const char *> optv(opts, opts + sizeof(opts) / sizeof(opts[0]));
    if (no_licm) {
        optv.push_back("-mllvm");
        optv.push_back("-disable-machine-licm");
    }
    const int preload = tuning().kernarg_preload;
    const std::string preload_opt = "-amdgpu-kernarg-preload-count=" + std::to_string(preload);
    if (preload > 0) {
        optv.push_back("-mllvm");
        optv.push_back(preload_opt.c_str());
    }
    hiprtcResult rc = hiprtcCompileProgram(prog, (int)optv.size(), optv.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        *error = std::string("hiprtc compile failed: ") + hiprtcGetErrorString(rc) + "\n" + log;
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    code->resize(code_size);
    hiprtcGetCode(prog, code->data());
    hiprtcDestroyProgram(&prog);
    return true;
}
}  // namespace

bool jit_compile(const Model &m, JitKind kind, bool f64, bool fast, const std::string &arch,
                 std::vector<char> *code, std::string *error, int pack, int tail, int nt, std::string *final_src) {
    std::string src = jit_source(m, kind, f64, fast, pack, tail, nt);
    // The paired fp32 rollout and the fp64 rollout of short chains keep 2 waves/SIMD only
    // without machine LICM: hoisting per-step address arithmetic and constants out of the K
    // loop costs the VGPRs below 256 (fp64 FR3: 212 instead of 264).
    const bool no_licm = kind == JitKind::Rollout && jit_rollout_no_hoist(f64, m.n, pack > 0 ? pack : jit_pack(kind, f64, m.n));
    if (!rtc_compile(src, arch, no_licm, code, error)) return false;
    // Occupancy cliff (jit.hpp): no target asked for, none in the source, and the kernel just
    // past 256 registers -> rebuild with a 2-wave target; the first build stands if that fails.
    if (tuning().jit_waves < 0 && src.find("amdgpu_waves_per_eu") == std::string::npos) {
        const int v = code_vgprs(*code);
        if (v > 256 && v <= 272) {
            std::string src2 = jit_source(m, kind, f64, fast, pack, tail, nt, 2), err2;
            std::vector<char> code2;
            if (rtc_compile(src2, arch, no_licm, &code2, &err2)) {
                code->swap(code2);
                src.swap(src2);
            }
        }
    }
    if (final_src) *final_src = src;
    // RB_JIT_DUMP=dir: keep every compiled source and code object for inspection
    // (llvm-objdump / llvm-readelf on the .co: registers, scratch, ISA of what really runs)
    if (const char *dir = std::getenv("RB_JIT_DUMP")) {
        static std::atomic<int> seq{0};
        const std::string base = std::string(dir) + "/jit_" + std::to_string(seq.fetch_add(1)) + "_k" +
                                 std::to_string((int)kind) + (f64 ? "_f64" : "_f32") + "_p" + std::to_string(pack);
        if (FILE *f = std::fopen((base + ".hip").c_str(), "wb")) {
            std::fwrite(src.data(), 1, src.size(), f);
            std::fclose(f);
        }
        if (FILE *f = std::fopen((base + ".co").c_str(), "wb")) {
            std::fwrite(code->data(), 1, code->size(), f);
            std::fclose(f);
        }
    }
    return true;
}

JitKernel jit_build(const Model &m, JitKind kind, bool f64, bool fast, int pack, int tail, int nt) {
    JitKernel jk;
    jk.pack = jit_model_pack(m, kind, f64, pack);
    if (kind == JitKind::Rnea && jk.pack == 3) jk.seq_tail = tail > 0 ? tail : 0;
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) {
        jk.error = "no HIP device";
        return jk;
    }
    std::vector<char> code;
    if (!jit_compile(m, kind, f64, fast, prop.gcnArchName, &code, &jk.error, jk.pack, jk.seq_tail, nt)) return jk;
    hipError_t e = hipModuleLoadData(&jk.module, code.data());
    if (e != hipSuccess) {
        jk.error = std::string("hipModuleLoadData: ") + hipGetErrorString(e);
        jk.module = nullptr;
        return jk;
    }
    e = hipModuleGetFunction(&jk.function, jk.module, "rb_jit_kernel");
    if (e != hipSuccess) {
        jk.error = std::string("hipModuleGetFunction: ") + hipGetErrorString(e);
        (void)hipModuleUnload(jk.module);
        jk.module = nullptr;
        jk.function = nullptr;
        return jk;
    }
    return jk;
}

}  // namespace rbamd
