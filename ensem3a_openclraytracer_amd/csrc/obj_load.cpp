// Native OBJ import with the reference importer's semantics (include/rt_scene.h).
//
// Reproduces FileManager.Scene's parse (FileManager.py:253-304) byte for byte:
//   * v / vn / vt lines anywhere in the file fill V_p / V_n / V_uv in file order
//     (the reference reads them through pywavefront: whitespace-separated
//     fields, decimal text -> double -> float32);
//   * lines before the first line whose first space-separated field is exactly
//     "usemtl" are otherwise ignored (faces there are lost);
//   * after it, a line starting with 'f' is one triangle "f p/uv/n p/uv/n p/uv/n"
//     (fields split on single spaces, only the first three vertices, 1-based
//     indices made 0-based), stored [mat, uv0..2, n0..2, p0..2]
//     (FileManager.py:276-282);
//   * any other line starting with 'u' increments the material counter.
// A face field the reference's int() would reject makes the parse fail.
#include <charconv>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/rt_scene.h"

struct rt_obj {
    std::vector<float> vp, vn, vuv;
    std::vector<int32_t> face;
    int64_t mat_counter = 0;
};

namespace {

thread_local std::string g_obj_error;

int fail(const std::string& msg) {
    g_obj_error = msg;
    return 1;
}

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// Python float(): the whole field must be a number (surrounding whitespace is already split off);
// correctly rounded like Python's, via std::from_chars (which takes no leading '+').
bool parse_float(const char* b, const char* e, double* out) {
    if (b == e) return false;
    const char* p = (*b == '+' && e - b > 1 && b[1] != '-' && b[1] != '+') ? b + 1 : b;
    const auto r = std::from_chars(p, e, *out, std::chars_format::general);
    if (r.ec == std::errc::result_out_of_range) {   // Python: huge literals -> +-inf, tiny -> +-0
        const std::string s(b, e);
        *out = std::strtod(s.c_str(), nullptr);
        return true;
    }
    return r.ec == std::errc() && r.ptr == e;
}

// Python int() on a field: optional surrounding whitespace, optional sign, decimal digits.
bool parse_int(const char* b, const char* e, long long* out) {
    while (b < e && is_space(*b)) ++b;
    while (e > b && is_space(e[-1])) --e;
    if (b == e) return false;
    bool neg = false;
    if (*b == '+' || *b == '-') neg = *b++ == '-';
    if (b == e) return false;
    long long v = 0;
    bool big = false;   // beyond 2^32: no int32 faceData entry can hold it
    for (const char* q = b; q < e; ++q) {
        if (*q < '0' || *q > '9') return false;
        if (!big) v = v * 10 + (*q - '0');
        big = big || v > (1ll << 32);
    }
    *out = big ? (neg ? -(1ll << 40) : (1ll << 40)) : (neg ? -v : v);
    return true;
}

// Whitespace-separated fields of [b, e).
void split_ws(const char* b, const char* e, std::vector<std::pair<const char*, const char*>>& f) {
    f.clear();
    const char* p = b;
    while (p < e) {
        while (p < e && is_space(*p)) ++p;
        if (p == e) break;
        const char* s = p;
        while (p < e && !is_space(*p)) ++p;
        f.emplace_back(s, p);
    }
}

}  // namespace

extern "C" {

const char* rt_obj_last_error(void) { return g_obj_error.c_str(); }

static int obj_parse(const char* text, int64_t len, rt_obj** out);

// No C++ exception leaves the C ABI: a file too large for host memory is a parse failure.
int rt_obj_parse(const char* text, int64_t len, rt_obj** out) {
    try {
        return obj_parse(text, len, out);
    } catch (const std::bad_alloc&) {
        return fail("out of host memory");
    }
}

static int obj_parse(const char* text, int64_t len, rt_obj** out) {
    if (!out || (!text && len > 0) || len < 0) return fail("bad arguments");
    *out = nullptr;
    std::unique_ptr<rt_obj> o(new rt_obj());   // freed on every failure path, and on bad_alloc
    std::vector<std::pair<const char*, const char*>> ws;
    bool seen_usemtl = false;
    const char* p = text;
    const char* end = text + len;
    int64_t lineno = 0;
    while (p < end) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        const char* le = nl ? nl + 1 : end;   // the line including its '\n', as Python iterates it
        ++lineno;
        split_ws(p, le, ws);
        if (!ws.empty()) {
            const size_t hl = (size_t)(ws[0].second - ws[0].first);
            const char* hp = ws[0].first;
            const bool is_v = hl == 1 && hp[0] == 'v';
            const bool is_vn = hl == 2 && hp[0] == 'v' && hp[1] == 'n';
            const bool is_vt = hl == 2 && hp[0] == 'v' && hp[1] == 't';
            if (is_v || is_vn) {
                if (ws.size() < 4) { return fail("line " + std::to_string(lineno) + ": short vertex"); }
                for (int k = 1; k <= 3; ++k) {
                    double v;
                    if (!parse_float(ws[k].first, ws[k].second, &v)) {
                        return fail("line " + std::to_string(lineno) + ": bad number");
                    }
                    (is_v ? o->vp : o->vn).push_back((float)v);
                }
            } else if (is_vt) {
                double u = 0.0, v = 0.0;
                if (ws.size() < 2 || !parse_float(ws[1].first, ws[1].second, &u) ||
                    (ws.size() > 2 && !parse_float(ws[2].first, ws[2].second, &v))) {
                    return fail("line " + std::to_string(lineno) + ": bad texture coordinate");
                }
                o->vuv.push_back((float)u);
                o->vuv.push_back((float)v);
            }
        }
        if (!seen_usemtl) {
            // line.split(" ")[0] == "usemtl"
            const char* sp = static_cast<const char*>(std::memchr(p, ' ', (size_t)(le - p)));
            const char* fe = sp ? sp : le;
            if (fe - p == 6 && std::memcmp(p, "usemtl", 6) == 0) seen_usemtl = true;
            p = le;
            continue;
        }
        if (*p == 'f') {
            // parts = line.split(" "); parts[1..3] = "p/uv/n"
            const char* fields[5];
            const char* fends[5];
            int nf = 0;
            const char* q = p;
            while (nf < 5) {
                const char* sp = static_cast<const char*>(std::memchr(q, ' ', (size_t)(le - q)));
                fields[nf] = q;
                fends[nf] = sp ? sp : le;
                ++nf;
                if (!sp) break;
                q = sp + 1;
            }
            if (nf < 4) { return fail("line " + std::to_string(lineno) + ": face with fewer than 3 vertices"); }
            int32_t row[10];
            row[0] = (int32_t)o->mat_counter;
            const int comps[3] = {1, 2, 0};   // uv, normal, position
            int w = 1;
            for (int ci = 0; ci < 3; ++ci) {
                for (int j = 1; j <= 3; ++j) {
                    // field.split("/")[comp]
                    const char* s = fields[j];
                    const char* fe = fends[j];
                    for (int skip = 0; skip < comps[ci]; ++skip) {
                        const char* sl = static_cast<const char*>(std::memchr(s, '/', (size_t)(fe - s)));
                        if (!sl) { return fail("line " + std::to_string(lineno) + ": face vertex without uv/normal"); }
                        s = sl + 1;
                    }
                    const char* sl = static_cast<const char*>(std::memchr(s, '/', (size_t)(fe - s)));
                    long long v;
                    if (!parse_int(s, sl ? sl : fe, &v)) {
                        return fail("line " + std::to_string(lineno) + ": bad face index");
                    }
                    // the reference stores faceData as int32 (FileManager.py:276-282): an index it cannot hold
                    // is refused here rather than wrapped
                    if (v - 1 < INT32_MIN || v - 1 > INT32_MAX) {
                        return fail("line " + std::to_string(lineno) + ": face index out of the int32 range");
                    }
                    row[w++] = (int32_t)(v - 1);
                }
            }
            o->face.insert(o->face.end(), row, row + 10);
        } else if (*p == 'u') {
            ++o->mat_counter;
        }
        p = le;
    }
    *out = o.release();
    return 0;
}

int64_t rt_obj_size(const rt_obj* o, int what) {
    if (!o) return -1;
    switch (what) {
        case RT_OBJ_VP: return (int64_t)o->vp.size();
        case RT_OBJ_VN: return (int64_t)o->vn.size();
        case RT_OBJ_VUV: return (int64_t)o->vuv.size();
        case RT_OBJ_FACE: return (int64_t)o->face.size();
        case RT_OBJ_MATERIALS: return o->mat_counter;
        default: return -1;
    }
}

int rt_obj_copy(const rt_obj* o, float* vp, float* vn, float* vuv, int32_t* face) {
    if (!o) return fail("null handle");
    if (vp && !o->vp.empty()) std::memcpy(vp, o->vp.data(), o->vp.size() * sizeof(float));
    if (vn && !o->vn.empty()) std::memcpy(vn, o->vn.data(), o->vn.size() * sizeof(float));
    if (vuv && !o->vuv.empty()) std::memcpy(vuv, o->vuv.data(), o->vuv.size() * sizeof(float));
    if (face && !o->face.empty()) std::memcpy(face, o->face.data(), o->face.size() * sizeof(int32_t));
    return 0;
}

void rt_obj_free(rt_obj* o) { delete o; }

}  // extern "C"
