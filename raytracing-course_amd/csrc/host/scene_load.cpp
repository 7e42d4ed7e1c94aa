// scene_load.cpp -- hw5 scene-file parser (drop-in for Scene::Load,
// /root/reference/hw5/src/sceneload.cpp:8-176).
//
// One pass over the file bytes, no per-line allocation.  It keeps the
// reference's observable behaviour, which is that of std::getline +
// std::stringstream extraction:
//  * lines split on '\n'; tokens on C-locale whitespace;
//  * a primitive block (after NEW_PRIMITIVE) ends at a blank line or at the
//    first non-primitive command; that command is then re-dispatched against
//    the *stale* NEW_PRIMITIVE line's stream (sceneload.cpp:120-159), so its
//    arguments are not read (values stay as they were);
//  * a failed numeric extraction stores 0 and poisons the rest of the line;
//    reading past the end of a line leaves the value unchanged;
//  * a primitive-type line (PLANE/BOX/ELLIPSOID/TRIANGLE) resets the whole
//    primitive (`primitive = Primitive(...)`, sceneload.cpp:49-72);
//  * unknown top-level commands warn on stderr (sceneload.cpp:170-172).
#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "pt_scene.h"

namespace pth {
namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }
inline bool is_dig(char c) { return c >= '0' && c <= '9'; }

// Decimal -> float for the common token (Clinger's fast path): with the decimal
// significand w <= 2^24 and the power of ten 10^|q| <= 10^10 both exact floats, ONE
// IEEE multiply or divide gives the correctly rounded value -- strtof's result (glibc
// strtof rounds correctly).  Tokens outside it go to strtof.  [b, e) is a scanned
// token: sign, digits, optional '.', digits, optional exponent, with at least one digit.
inline bool fast_float(const char* b, const char* e, float& out) {
    static const float p10[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
    const char* c = b;
    bool neg = false;
    if (*c == '+' || *c == '-') neg = *c++ == '-';
    uint64_t w = 0;
    int nd = 0, q = 0;
    for (; c < e && is_dig(*c); ++c) {
        if (w || *c != '0') { if (++nd > 9) return false; w = w * 10u + (uint64_t)(*c - '0'); }
    }
    if (c < e && *c == '.') {
        for (++c; c < e && is_dig(*c); ++c) {
            --q;
            if (w || *c != '0') { if (++nd > 9) return false; w = w * 10u + (uint64_t)(*c - '0'); }
        }
    }
    if (c < e) {   // exponent
        ++c;
        bool eneg = false;
        if (c < e && (*c == '+' || *c == '-')) eneg = *c++ == '-';
        if (c == e) return false;   // "1e" / "1e+": strtof decides (the token then fails)
        int x = 0;
        for (; c < e; ++c) {
            if (x > 1000) return false;
            x = x * 10 + (*c - '0');
        }
        q += eneg ? -x : x;
    }
    if (w > (1u << 24)) return false;
    float f;
    if (w == 0) f = 0.f;
    else if (q >= 0 && q <= 10) f = (float)w * p10[q];
    else if (q < 0 && q >= -10) f = (float)w / p10[-q];
    else return false;
    out = neg ? -f : f;
    return true;
}

// the remainder of one line, read like a std::stringstream
struct Cursor {
    const char* p;
    const char* e;
    bool fail = false;
    Cursor(const char* b, const char* en) : p(b), e(en) {}
    void skip() { while (p < e && is_ws(*p)) ++p; }
    // operator>>(std::string&)
    bool word(const char*& wb, size_t& wl) {
        if (fail) return false;
        skip();
        if (p >= e) { fail = true; return false; }
        wb = p;
        while (p < e && !is_ws(*p)) ++p;
        wl = (size_t)(p - wb);
        return true;
    }
    // operator>>(float&)  (num_get::_M_extract_float + strtof)
    void get(float& v) {
        if (fail) return;
        skip();
        if (p >= e) { fail = true; return; }
        const char* b = p;
        const char* q = p;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        bool dig = false;
        while (q < e && is_dig(*q)) { ++q; dig = true; }
        if (q < e && *q == '.') { ++q; while (q < e && is_dig(*q)) { ++q; dig = true; } }
        if (dig && q < e && (*q == 'e' || *q == 'E')) {
            const char* r = q + 1;
            if (r < e && (*r == '+' || *r == '-')) ++r;
            if (r < e && is_dig(*r)) { while (r < e && is_dig(*r)) ++r; }
            q = r;
        }
        p = q;
        const size_t n = (size_t)(q - b);
        if (dig && fast_float(b, q, v)) return;
        char buf[128];
        if (n == 0 || n >= sizeof(buf)) { v = 0.f; fail = true; return; }
        memcpy(buf, b, n);
        buf[n] = '\0';
        char* end = nullptr;
        const float f = strtof(buf, &end);
        if (end != buf + n) { v = 0.f; fail = true; return; }
        v = f;
    }
    // operator>>(unsigned&)
    void get(uint32_t& v) {
        if (fail) return;
        skip();
        if (p >= e) { fail = true; return; }
        bool neg = false;
        if (*p == '+' || *p == '-') { neg = *p == '-'; ++p; }
        const char* d0 = p;
        unsigned long long acc = 0;
        bool ovf = false;
        while (p < e && is_dig(*p)) {
            acc = acc * 10 + (unsigned)(*p - '0');
            if (acc > 0xFFFFFFFFull) ovf = true;
            ++p;
        }
        if (p == d0) { v = 0; fail = true; return; }
        if (ovf) { v = 0xFFFFFFFFu; fail = true; return; }
        v = neg ? (uint32_t)(0u - (uint32_t)acc) : (uint32_t)acc;
    }
    void get3(float* x) { get(x[0]); get(x[1]); get(x[2]); }
};

enum Cmd {
    C_EMPTY, C_DIMENSIONS, C_BG_COLOR, C_CAMERA_POSITION, C_CAMERA_RIGHT, C_CAMERA_UP, C_CAMERA_FORWARD,
    C_CAMERA_FOV_X, C_NEW_PRIMITIVE, C_PLANE, C_ELLIPSOID, C_BOX, C_POSITION, C_ROTATION, C_COLOR,
    C_RAY_DEPTH, C_METALLIC, C_DIELECTRIC, C_IOR, C_SAMPLES, C_EMISSION, C_TRIANGLE, C_UNKNOWN
};

// src/sceneload.cpp:8-33
Cmd command_of(const char* w, size_t n) {
    if (n == 0) return C_EMPTY;
    struct E { const char* s; Cmd c; };
    static const E tab[] = {
        {"DIMENSIONS", C_DIMENSIONS}, {"BG_COLOR", C_BG_COLOR}, {"CAMERA_POSITION", C_CAMERA_POSITION},
        {"CAMERA_RIGHT", C_CAMERA_RIGHT}, {"CAMERA_UP", C_CAMERA_UP}, {"CAMERA_FORWARD", C_CAMERA_FORWARD},
        {"CAMERA_FOV_X", C_CAMERA_FOV_X}, {"NEW_PRIMITIVE", C_NEW_PRIMITIVE}, {"PLANE", C_PLANE},
        {"ELLIPSOID", C_ELLIPSOID}, {"BOX", C_BOX}, {"POSITION", C_POSITION}, {"ROTATION", C_ROTATION},
        {"COLOR", C_COLOR}, {"RAY_DEPTH", C_RAY_DEPTH}, {"METALLIC", C_METALLIC}, {"DIELECTRIC", C_DIELECTRIC},
        {"IOR", C_IOR}, {"SAMPLES", C_SAMPLES}, {"EMISSION", C_EMISSION}, {"TRIANGLE", C_TRIANGLE}};
    for (const E& x : tab)
        if (strlen(x.s) == n && memcmp(x.s, w, n) == 0) return x.c;
    return C_UNKNOWN;
}

struct Lines {
    const char* p;
    const char* e;
    bool next(const char*& lb, const char*& le) {
        if (p >= e) return false;
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(e - p)));
        lb = p;
        le = nl ? nl : e;
        p = nl ? nl + 1 : e;
        return true;
    }
};

inline void reset_prim(HPrim& pr, uint32_t type) { pr = HPrim(); pr.type = type; }

// src/sceneload.cpp:35-110; returns the command that ended the block ("" = blank line / EOF)
std::string load_primitive(Lines& L, HPrim& pr) {
    const char *lb, *le;
    while (L.next(lb, le)) {
        Cursor ss(lb, le);
        const char* w = nullptr;
        size_t wl = 0;
        ss.word(w, wl);
        const Cmd cmd = command_of(w, wl);
        if (cmd == C_EMPTY) break;
        switch (cmd) {
            case C_ELLIPSOID: { float r[3] = {0, 0, 0}; ss.get3(r); reset_prim(pr, pt::T_ELLIPSOID); memcpy(pr.a, r, 12); break; }
            case C_PLANE: { float n[3] = {0, 0, 0}; ss.get3(n); reset_prim(pr, pt::T_PLANE); memcpy(pr.a, n, 12); break; }
            case C_BOX: { float s[3] = {0, 0, 0}; ss.get3(s); reset_prim(pr, pt::T_BOX); memcpy(pr.a, s, 12); break; }
            case C_TRIANGLE: {
                float a[3] = {0, 0, 0}, b[3] = {0, 0, 0}, c[3] = {0, 0, 0};
                ss.get3(a); ss.get3(b); ss.get3(c);
                reset_prim(pr, pt::T_TRIANGLE);
                memcpy(pr.a, a, 12); memcpy(pr.b, b, 12); memcpy(pr.c, c, 12);
                break;
            }
            case C_COLOR: ss.get3(pr.col); break;
            case C_POSITION: ss.get3(pr.pos); break;
            case C_ROTATION: ss.get(pr.rot[0]); ss.get(pr.rot[1]); ss.get(pr.rot[2]); ss.get(pr.rot[3]); break;
            case C_METALLIC: pr.mat = pt::M_METALLIC; break;
            case C_DIELECTRIC: pr.mat = pt::M_DIELECTRIC; break;
            case C_IOR: ss.get(pr.ior); break;
            case C_EMISSION: ss.get3(pr.emis); break;
            default: return std::string(w, wl);
        }
    }
    return std::string();
}

// a top-level command (src/sceneload.cpp:114-172) on its line's stream `ss` (for a
// command that ended a primitive block: the stale NEW_PRIMITIVE line's stream)
void top_level(HScene& S, Cmd cmd, const std::string& name, Cursor& ss) {
    switch (cmd) {
        case C_DIMENSIONS: ss.get(S.W); ss.get(S.H); break;
        case C_BG_COLOR: ss.get3(S.bg); break;
        case C_CAMERA_POSITION: ss.get3(S.cam_pos); break;
        case C_CAMERA_RIGHT: ss.get3(S.cam_right); break;
        case C_CAMERA_UP: ss.get3(S.cam_up); break;
        case C_CAMERA_FORWARD: ss.get3(S.cam_fwd); break;
        case C_CAMERA_FOV_X: ss.get(S.fov_x); break;
        case C_RAY_DEPTH: ss.get(S.depth); break;
        case C_SAMPLES: ss.get(S.samples); break;
        default: {
            fprintf(stderr, "unexpected command(%s)\n", name.c_str());
            S.warnings.push_back("unexpected command(" + name + ")");
            break;
        }
    }
}

// One stretch of the file: its primitives, and its top-level commands with their
// streams, in order (replayed on the scene after every stretch is parsed, since
// a command's effect can depend on the values before it: a failed extraction keeps them)
struct Event {
    Cmd cmd;
    std::string name;
    Cursor ss;
};
struct Stretch {
    std::vector<HPrim> prims;
    std::vector<Event> events;
};

// src/sceneload.cpp:112-176 over [text, text + len)
void parse_stretch(const char* text, size_t len, Stretch& out) {
    Lines L{text, text + len};
    const char *lb, *le;
    std::string name;
    while (L.next(lb, le)) {
        Cursor ss(lb, le);
        const char* w = nullptr;
        size_t wl = 0;
        ss.word(w, wl);
        name.assign(w ? w : "", w ? wl : 0);
    again:
        const Cmd cmd = command_of(name.data(), name.size());
        if (cmd == C_EMPTY) continue;
        if (cmd == C_NEW_PRIMITIVE) {
            HPrim pr;
            name = load_primitive(L, pr);
            out.prims.push_back(pr);
            if (!name.empty()) goto again;   // the stale `ss` is reused, as in the reference
            continue;
        }
        out.events.push_back(Event{cmd, name, ss});
    }
}

// does the line at p (up to e) start with the token NEW_PRIMITIVE (stringstream >> skips
// leading whitespace)?
bool starts_new_primitive(const char* p, const char* e) {
    while (p < e && *p != '\n' && is_ws(*p)) ++p;
    static const char k[] = "NEW_PRIMITIVE";
    const size_t n = sizeof(k) - 1;
    return (size_t)(e - p) >= n && memcmp(p, k, n) == 0 && (p + n == e || is_ws(p[n]));
}

}  // namespace

// src/sceneload.cpp:112-176.  A large file is parsed in stretches on several threads.
// A line whose first token is NEW_PRIMITIVE always starts a new primitive after pushing
// the one being read -- at the top level, and inside a block too (load_primitive returns
// it, and the top level dispatches it; NEW_PRIMITIVE reads nothing from the stale
// stream) -- so stretches that begin at such lines parse independently.  Their
// primitives are concatenated in order, and their top-level commands replayed in order.
void parse_scene(const char* text, size_t len, HScene& S) {
    unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (len < (1u << 20)) T = 1;
    std::vector<size_t> cut{0};
    for (unsigned k = 1; k < T; ++k) {
        size_t at = std::max(cut.back(), len * k / T);
        // the next line start at or after `at` whose line begins a primitive
        if (at > 0) {
            const void* nl = memchr(text + at - 1, '\n', len - (at - 1));
            at = nl ? (size_t)(static_cast<const char*>(nl) - text) + 1 : len;
        }
        while (at < len && !starts_new_primitive(text + at, text + len)) {
            const void* nl = memchr(text + at, '\n', len - at);
            at = nl ? (size_t)(static_cast<const char*>(nl) - text) + 1 : len;
        }
        if (at >= len) break;
        if (at > cut.back()) cut.push_back(at);
    }
    cut.push_back(len);
    const size_t n = cut.size() - 1;
    std::vector<Stretch> parts(n);
    if (n == 1) {
        parse_stretch(text, len, parts[0]);
    } else {
        // (a stretch whose thread cannot be started is parsed here, after the others start)
        std::vector<std::thread> th;
        std::vector<size_t> here;
        for (size_t i = 0; i < n; ++i) {
            try {
                th.emplace_back([&, i] { parse_stretch(text + cut[i], cut[i + 1] - cut[i], parts[i]); });
            } catch (const std::system_error&) {
                here.push_back(i);
            }
        }
        for (size_t i : here) parse_stretch(text + cut[i], cut[i + 1] - cut[i], parts[i]);
        for (auto& t : th) t.join();
    }
    size_t np = 0;
    for (const auto& p : parts) np += p.prims.size();
    S.prims.reserve(S.prims.size() + np);
    for (auto& p : parts) {
        S.prims.insert(S.prims.end(), p.prims.begin(), p.prims.end());
        for (auto& ev : p.events) top_level(S, ev.cmd, ev.name, ev.ss);
    }
}

}  // namespace pth
