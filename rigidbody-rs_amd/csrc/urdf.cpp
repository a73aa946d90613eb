// urdf.cpp -- see urdf.hpp.
#include "urdf.hpp"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace rbamd {

const char *XmlNode::attr(const char *name) const {
    for (const auto &kv : attrs)
        if (kv.first == name) return kv.second.c_str();
    return nullptr;
}

const XmlNode *XmlNode::child(const char *t) const {
    for (const auto &c : children)
        if (c.tag == t) return &c;
    return nullptr;
}

namespace {

// Nesting limit: element() recurses per level, so an adversarial document of deeply nested
// tags would otherwise exhaust the stack (URDFs nest 4-5 levels).
constexpr int kMaxDepth = 256;

struct Parser {
    const std::string &s;
    size_t i = 0;
    int depth = 0;

    [[noreturn]] void fail(const char *what) const {
        throw std::runtime_error(std::string("XML parse error at offset ") + std::to_string(i) +
                                 ": " + what);
    }
    bool starts(const char *p) const { return s.compare(i, std::strlen(p), p) == 0; }
    void skip_ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    void skip_until(const char *end) {
        size_t j = s.find(end, i);
        if (j == std::string::npos) fail("unterminated construct");
        i = j + std::strlen(end);
    }
    // Skips comments, processing instructions, doctype and text between elements.
    void skip_misc() {
        for (;;) {
            while (i < s.size() && s[i] != '<') ++i;  // text content is not needed
            if (i >= s.size()) return;
            if (starts("<!--")) { skip_until("-->"); continue; }
            if (starts("<?")) { skip_until("?>"); continue; }
            if (starts("<![CDATA[")) { skip_until("]]>"); continue; }
            if (starts("<!")) { skip_until(">"); continue; }
            return;
        }
    }
    std::string name() {
        size_t b = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_' || s[i] == '-' ||
                                s[i] == ':' || s[i] == '.'))
            ++i;
        if (b == i) fail("expected a name");
        return s.substr(b, i - b);
    }
    static std::string unescape(const std::string &v) {
        std::string o;
        o.reserve(v.size());
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] == '&') {
                size_t e = v.find(';', k);
                if (e != std::string::npos) {
                    std::string ent = v.substr(k + 1, e - k - 1);
                    if (ent == "lt") { o += '<'; k = e; continue; }
                    if (ent == "gt") { o += '>'; k = e; continue; }
                    if (ent == "amp") { o += '&'; k = e; continue; }
                    if (ent == "quot") { o += '"'; k = e; continue; }
                    if (ent == "apos") { o += '\''; k = e; continue; }
                }
            }
            o += v[k];
        }
        return o;
    }
    XmlNode element() {
        if (i >= s.size() || s[i] != '<') fail("expected '<'");
        if (++depth > kMaxDepth) fail("elements nested too deeply");
        ++i;
        XmlNode n;
        n.tag = name();
        for (;;) {
            skip_ws();
            if (i >= s.size()) fail("unterminated start tag");
            if (starts("/>")) { i += 2; --depth; return n; }
            if (s[i] == '>') { ++i; break; }
            std::string k = name();
            skip_ws();
            if (i >= s.size() || s[i] != '=') fail("expected '=' after attribute name");
            ++i;
            skip_ws();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) fail("expected quoted attribute");
            char q = s[i++];
            size_t e = s.find(q, i);
            if (e == std::string::npos) fail("unterminated attribute value");
            n.attrs.emplace_back(k, unescape(s.substr(i, e - i)));
            i = e + 1;
        }
        for (;;) {
            skip_misc();
            if (i >= s.size()) fail("unterminated element");
            if (starts("</")) {
                i += 2;
                std::string close = name();
                if (close != n.tag) fail("mismatched closing tag");
                skip_ws();
                if (i >= s.size() || s[i] != '>') fail("expected '>'");
                ++i;
                --depth;
                return n;
            }
            n.children.push_back(element());
        }
    }
};

void parse_numbers(const char *text, double *out, int n, const char *what) {
    if (!text) return;  // attribute absent: keep defaults
    const char *p = text;
    for (int k = 0; k < n; ++k) {
        char *end = nullptr;
        double v = std::strtod(p, &end);
        if (end == p) throw std::runtime_error(std::string("bad number list in ") + what);
        if (!std::isfinite(v)) throw std::runtime_error(std::string("non-finite number in ") + what);
        out[k] = v;
        p = end;
    }
    while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') ++p;
    if (*p) throw std::runtime_error(std::string("too many numbers in ") + what);
}

double parse_one(const char *text, const char *what) {
    double v = 0.0;
    parse_numbers(text, &v, 1, what);
    return v;
}

}  // namespace

XmlNode parse_xml(const std::string &text) {
    Parser p{text};
    p.skip_misc();
    XmlNode root = p.element();
    return root;
}

UrdfRobot parse_urdf(const std::string &text) {
    XmlNode root = parse_xml(text);
    if (root.tag != "robot") throw std::runtime_error("URDF root element is not <robot>");
    UrdfRobot r;
    if (const char *nm = root.attr("name")) r.name = nm;
    for (const XmlNode &el : root.children) {
        if (el.tag == "link") {
            UrdfLink L;
            if (const char *nm = el.attr("name")) L.name = nm;
            if (const XmlNode *in = el.child("inertial")) {
                if (const XmlNode *o = in->child("origin")) {
                    parse_numbers(o->attr("xyz"), L.com, 3, "inertial origin xyz");
                    parse_numbers(o->attr("rpy"), L.com_rpy, 3, "inertial origin rpy");
                }
                if (const XmlNode *m = in->child("mass")) L.mass = parse_one(m->attr("value"), "mass");
                if (const XmlNode *t = in->child("inertia")) {
                    static const char *keys[6] = {"ixx", "ixy", "ixz", "iyy", "iyz", "izz"};
                    for (int k = 0; k < 6; ++k)
                        if (const char *v = t->attr(keys[k])) L.inertia6[k] = parse_one(v, keys[k]);
                }
            }
            r.links.push_back(L);
        } else if (el.tag == "joint") {
            UrdfJoint J;
            if (const char *nm = el.attr("name")) J.name = nm;
            if (const char *ty = el.attr("type")) J.type = ty;
            if (const XmlNode *o = el.child("origin")) {
                parse_numbers(o->attr("xyz"), J.xyz, 3, "joint origin xyz");
                parse_numbers(o->attr("rpy"), J.rpy, 3, "joint origin rpy");
            }
            if (const XmlNode *a = el.child("axis")) parse_numbers(a->attr("xyz"), J.axis, 3, "axis");
            if (const XmlNode *p = el.child("parent")) if (const char *v = p->attr("link")) J.parent = v;
            if (const XmlNode *c = el.child("child")) if (const char *v = c->attr("link")) J.child = v;
            J.mimic = el.child("mimic") != nullptr;
            if (const XmlNode *l = el.child("limit")) {
                if (const char *v = l->attr("lower")) J.lower = parse_one(v, "limit lower");
                if (const char *v = l->attr("upper")) J.upper = parse_one(v, "limit upper");
                if (const char *v = l->attr("effort")) J.effort = parse_one(v, "limit effort");
                if (const char *v = l->attr("velocity")) J.velocity = parse_one(v, "limit velocity");
            }
            r.joints.push_back(J);
        }
    }
    return r;
}

std::vector<RawJoint> select_chain(const UrdfRobot &robot, bool *pairing_matches_child) {
    std::vector<RawJoint> out;
    bool match = true;
    size_t n = robot.joints.size() < robot.links.size() ? robot.joints.size() : robot.links.size();
    for (size_t k = 0; k < n; ++k) {
        const UrdfJoint &j = robot.joints[k];
        if (j.type.find("fixed") != std::string::npos) continue;
        if (j.child != robot.links[k].name) match = false;
        out.push_back(RawJoint{j, robot.links[k]});
    }
    if (pairing_matches_child) *pairing_matches_child = match;
    return out;
}

}  // namespace rbamd
