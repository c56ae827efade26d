// omr_request.cpp — request decode and renderer settings of the drop-in (host only).
//
// The reference turns a Vert.x MultiMap into an ImageRegionCtx (ImageRegionCtx.java:127-402)
// and then pushes the ctx onto a fresh omeis Renderer (ImageRegionRequestHandler.java:689-741,
// updateSettings).  Both steps decide every kernel parameter of the render, so they are
// restated here with Java's parsing semantics:
//   Integer.parseInt / Long.parseLong / Float.parseFloat / Boolean.parseBoolean,
//   String.split(regex, limit) trailing-empty rules, Jackson's List decode of `maps`,
//   Guava sipHash24 cache key (ImageRegionCtx.java:165-177),
// and the exceptions the reference would throw become status codes:
//   IllegalArgumentException (incl. NumberFormatException) -> OMR_INVALID_ARGUMENT (400)
//   NullPointerException / ClassCastException / IndexOutOfBounds / DecodeException -> OMR_INTERNAL (500)
//
// LutProviderImpl (LutProviderImpl.java:29-75) is here too: it scans a root for *.lut files
// once and serves 768-byte R/G/B tables by basename.
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "omr/omr.h"

namespace {

// ---------------------------------------------------------------- Java string semantics
// String.split with a single literal delimiter (all the reference's regexes are literal:
// ",", "\\|", "\\$", ":").  limit < 0 keeps trailing empties, limit == 0 drops them,
// limit > 0 caps the number of parts.
std::vector<std::string> jsplit(const std::string& s, char d, int limit) {
    std::vector<std::string> out;
    size_t start = 0;
    for (;;) {
        if (limit > 0 && (int)out.size() == limit - 1) break;
        const size_t p = s.find(d, start);
        if (p == std::string::npos) break;
        out.push_back(s.substr(start, p - start));
        start = p + 1;
    }
    if (out.empty()) return {s};        // no match: the input itself
    out.push_back(s.substr(start));
    if (limit == 0)
        while (!out.empty() && out.back().empty()) out.pop_back();
    return out;
}

// Integer.parseInt / Long.parseLong (radix 10): optional sign, >= 1 ASCII digit, range-checked.
bool jparse_long(const std::string& s, int64_t lo, int64_t hi, int64_t& out) {
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        i = 1;
        if (s.size() == 1) return false;
    }
    // accumulate negatively like the JDK so that MIN_VALUE parses
    int64_t acc = 0;
    for (; i < s.size(); ++i) {
        const char c = s[i];
        if (c < '0' || c > '9') return false;
        const int d = c - '0';
        if (acc < (INT64_MIN + d) / 10) return false;
        acc = acc * 10 - d;
    }
    if (!neg) {
        if (acc == INT64_MIN) return false;
        acc = -acc;
    }
    if (acc < lo || acc > hi) return false;
    out = acc;
    return true;
}

bool jparse_int(const std::string& s, int32_t& out) {
    int64_t v;
    if (!jparse_long(s, INT32_MIN, INT32_MAX, v)) return false;
    out = (int32_t)v;
    return true;
}

// Float.parseFloat (FloatingDecimal.readJavaFormatString): trims chars <= ' ', optional sign,
// "NaN" / "Infinity", decimal digits with optional '.', exponent, and a trailing
// f/F/d/D type suffix; hexadecimal "0x1.8p3" forms.  Correctly rounded to float.
bool jparse_float(const std::string& raw, float& out) {
    size_t b = 0, e = raw.size();
    while (b < e && (unsigned char)raw[b] <= ' ') ++b;
    while (e > b && (unsigned char)raw[e - 1] <= ' ') --e;
    std::string s = raw.substr(b, e - b);
    if (s.empty()) return false;
    size_t i = 0;
    std::string sign;
    if (s[0] == '+' || s[0] == '-') { sign = s.substr(0, 1); i = 1; }
    const std::string body = s.substr(i);
    if (body == "NaN") { out = NAN; return true; }
    if (body == "Infinity") { out = sign == "-" ? -INFINITY : INFINITY; return true; }
    std::string num = body;
    if (!num.empty() && std::strchr("fFdD", num.back())) num.pop_back();
    if (num.empty()) return false;
    const bool hex = num.size() > 2 && num[0] == '0' && (num[1] == 'x' || num[1] == 'X');
    size_t k = hex ? 2 : 0;
    int mant = 0;
    auto isdig = [hex](char c) {
        return (c >= '0' && c <= '9') || (hex && ((c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F')));
    };
    while (k < num.size() && isdig(num[k])) { ++k; ++mant; }
    if (k < num.size() && num[k] == '.') {
        ++k;
        while (k < num.size() && isdig(num[k])) { ++k; ++mant; }
    }
    if (mant == 0) return false;
    const char ech = hex ? 'p' : 'e';
    if (k < num.size() && (num[k] == ech || num[k] == ech - 32)) {
        ++k;
        if (k < num.size() && (num[k] == '+' || num[k] == '-')) ++k;
        int ed = 0;
        while (k < num.size() && num[k] >= '0' && num[k] <= '9') { ++k; ++ed; }
        if (ed == 0) return false;
    } else if (hex) {
        return false;                 // Java requires the binary exponent on hex floats
    }
    if (k != num.size()) return false;
    const std::string full = sign + num;
    errno = 0;
    out = std::strtof(full.c_str(), nullptr);   // round-to-nearest-even, overflow -> +-inf like Java
    return true;
}

std::string lower(std::string s) {
    for (auto& c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

bool iequals(const std::string& a, const std::string& b) { return lower(a) == lower(b); }

// ---------------------------------------------------------------- Vert.x caseInsensitiveMultiMap
struct MultiMap {
    std::vector<std::pair<std::string, std::string>> entries;   // insertion order
    const std::string* get(const char* key) const {             // first value, case-insensitive
        for (auto& kv : entries)
            if (iequals(kv.first, key)) return &kv.second;
        return nullptr;
    }
    std::vector<std::string> names() const {                    // first-seen case per name
        std::vector<std::string> n;
        for (auto& kv : entries) {
            bool seen = false;
            for (auto& x : n) seen = seen || iequals(x, kv.first);
            if (!seen) n.push_back(kv.first);
        }
        return n;
    }
};

// ---------------------------------------------------------------- Guava Hashing.sipHash24()
inline uint64_t rotl(uint64_t x, int b) { return (x << b) | (x >> (64 - b)); }

uint64_t siphash24(const uint8_t* m, size_t n, uint64_t k0, uint64_t k1) {
    uint64_t v0 = 0x736f6d6570736575ull ^ k0, v1 = 0x646f72616e646f6dull ^ k1;
    uint64_t v2 = 0x6c7967656e657261ull ^ k0, v3 = 0x7465646279746573ull ^ k1;
    auto round = [&]() {
        v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
        v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
        v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
        v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
    };
    const size_t full = n / 8 * 8;
    for (size_t i = 0; i < full; i += 8) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w |= (uint64_t)m[i + j] << (8 * j);
        v3 ^= w; round(); round(); v0 ^= w;
    }
    uint64_t last = (uint64_t)(n & 0xFF) << 56;
    for (size_t j = 0; j < n - full; ++j) last |= (uint64_t)m[full + j] << (8 * j);
    v3 ^= last; round(); round(); v0 ^= last;
    v2 ^= 0xFF;
    round(); round(); round(); round();
    return v0 ^ v1 ^ v2 ^ v3;
}

// HashCode.fromLong(h).toString(): lower-case hex of the little-endian bytes.
void hash_hex(uint64_t h, char out[17]) {
    static const char* hx = "0123456789abcdef";
    for (int i = 0; i < 8; ++i) {
        const unsigned b = (unsigned)(h >> (8 * i)) & 0xFF;
        out[2 * i] = hx[b >> 4];
        out[2 * i + 1] = hx[b & 15];
    }
    out[16] = 0;
}

// ---------------------------------------------------------------- minimal JSON (Jackson List decode)
// Only what updateSettings reads is kept: per list element whether it is null / an object /
// something else, and for objects the "reverse" member's "enabled" value.
struct JsonCursor {
    const std::string& s;
    size_t i = 0;
    explicit JsonCursor(const std::string& str) : s(str) {}
    void ws() { while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i; }
    bool lit(const char* w) {
        const size_t n = std::strlen(w);
        if (s.compare(i, n, w) == 0) { i += n; return true; }
        return false;
    }
    bool string(std::string* out) {
        if (i >= s.size() || s[i] != '"') return false;
        ++i;
        std::string v;
        while (i < s.size() && s[i] != '"') {
            if ((unsigned char)s[i] < 0x20) return false;
            if (s[i] == '\\') {
                ++i;
                if (i >= s.size()) return false;
                const char c = s[i];
                if (c == 'u') {
                    if (i + 4 >= s.size()) return false;
                    for (int k = 1; k <= 4; ++k)
                        if (!std::isxdigit((unsigned char)s[i + k])) return false;
                    v += '?';
                    i += 5;
                    continue;
                }
                if (!std::strchr("\"\\/bfnrt", c)) return false;
                v += c == 'n' ? '\n' : c == 't' ? '\t' : c;
                ++i;
                continue;
            }
            v += s[i++];
        }
        if (i >= s.size()) return false;
        ++i;
        if (out) *out = v;
        return true;
    }
    bool number() {
        const size_t st = i;
        if (i < s.size() && s[i] == '-') ++i;
        if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return false;
        if (s[i] == '0') ++i;
        else while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        if (i < s.size() && s[i] == '.') {
            ++i;
            if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return false;
            while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        }
        if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
            ++i;
            if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
            if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return false;
            while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        }
        return i > st;
    }
    // kind: 0 null, 1 true, 2 false, 3 object, 4 other
    bool value(int* kind, int depth, int* reverse_state);
};

// reverse_state (objects only, depth 0 elements of the list):
//   OMR_MAP_NONE (no "reverse" member, or not enabled == TRUE), OMR_MAP_REVERSE,
//   OMR_MAP_BAD (the "reverse" member is present but not an object/null -> ClassCastException)
bool JsonCursor::value(int* kind, int depth, int* reverse_state) {
    if (depth > 64) return false;
    ws();
    if (i >= s.size()) return false;
    const char c = s[i];
    if (c == 'n') { if (!lit("null")) return false; *kind = 0; return true; }
    if (c == 't') { if (!lit("true")) return false; *kind = 1; return true; }
    if (c == 'f') { if (!lit("false")) return false; *kind = 2; return true; }
    if (c == '"') { *kind = 4; return string(nullptr); }
    if (c == '[') {
        ++i; ws();
        *kind = 4;
        if (i < s.size() && s[i] == ']') { ++i; return true; }
        for (;;) {
            int k;
            if (!value(&k, depth + 1, nullptr)) return false;
            ws();
            if (i < s.size() && s[i] == ',') { ++i; continue; }
            if (i < s.size() && s[i] == ']') { ++i; return true; }
            return false;
        }
    }
    if (c == '{') {
        ++i; ws();
        *kind = 3;
        if (reverse_state) *reverse_state = OMR_MAP_NONE;
        if (i < s.size() && s[i] == '}') { ++i; return true; }
        for (;;) {
            ws();
            std::string key;
            if (!string(&key)) return false;
            ws();
            if (i >= s.size() || s[i] != ':') return false;
            ++i;
            const bool is_reverse = reverse_state && key == "reverse";
            int k, inner = OMR_MAP_NONE;
            // the "reverse" member: an object whose "enabled" member is read
            if (is_reverse) {
                ws();
                if (i < s.size() && s[i] == '{') {
                    ++i; ws();
                    if (i < s.size() && s[i] == '}') { ++i; k = 3; }
                    else {
                        for (;;) {
                            ws();
                            std::string k2;
                            if (!string(&k2)) return false;
                            ws();
                            if (i >= s.size() || s[i] != ':') return false;
                            ++i;
                            int vk;
                            if (!value(&vk, depth + 2, nullptr)) return false;
                            // HashMap.put: a later duplicate key wins
                            if (k2 == "enabled") inner = vk == 1 ? OMR_MAP_REVERSE : OMR_MAP_NONE;
                            ws();
                            if (i < s.size() && s[i] == ',') { ++i; continue; }
                            if (i < s.size() && s[i] == '}') { ++i; break; }
                            return false;
                        }
                        k = 3;
                    }
                } else {
                    if (!value(&k, depth + 1, nullptr)) return false;
                    inner = k == 0 ? OMR_MAP_NONE : OMR_MAP_BAD;
                }
                *reverse_state = inner;
            } else if (!value(&k, depth + 1, nullptr)) {
                return false;
            }
            ws();
            if (i < s.size() && s[i] == ',') { ++i; continue; }
            if (i < s.size() && s[i] == '}') { ++i; return true; }
            return false;
        }
    }
    *kind = 4;
    return number();
}

void set_err(char* err, size_t cap, const std::string& msg) {
    if (!err || cap == 0) return;
    const size_t n = std::min(cap - 1, msg.size());
    std::memcpy(err, msg.data(), n);
    err[n] = 0;
}

void copy_str(char* dst, size_t cap, const std::string& s) {
    const size_t n = std::min(cap - 1, s.size());
    std::memcpy(dst, s.data(), n);
    dst[n] = 0;
}

// ImageRegionCtx.getChannelInfoFromString (:281-326) for one comma-separated entry.
bool parse_channel(const std::string& channel, omr_image_region_ctx* o, int idx) {
    const std::vector<std::string> temp = jsplit(channel, '|', 2);
    std::string active = temp[0];
    bool has_color = false;
    std::string color;
    bool has_window = false;
    std::string window;
    if (active.find('$') != std::string::npos) {
        const std::vector<std::string> sp = jsplit(active, '$', -1);
        active = sp[0];
        color = sp[1];
        has_color = true;
    }
    int32_t a;
    if (!jparse_int(active, a)) return false;
    o->channels[idx] = a;
    o->window_set[idx] = 0;
    o->windows[idx][0] = o->windows[idx][1] = 0.0f;
    if (temp.size() > 1) {
        if (temp[1].find('$') != std::string::npos) {
            const std::vector<std::string> sp = jsplit(temp[1], '$', 0);
            if (sp.empty()) return false;            // "$" alone: split -> [] -> [0] throws
            window = sp[0];
            has_window = true;
            if (sp.size() < 2) return false;         // ArrayIndexOutOfBounds -> IAE
            color = sp[1];
            has_color = true;
        }
        if (!has_window) return false;               // window.split on null -> NPE -> IAE
        const std::vector<std::string> range = jsplit(window, ':', 0);
        if (range.size() > 1) {
            float lo, hi;
            if (!jparse_float(range[0], lo) || !jparse_float(range[1], hi)) return false;
            o->windows[idx][0] = lo;
            o->windows[idx][1] = hi;
            o->window_set[idx] = 1;
        }
    }
    o->color_set[idx] = has_color ? 1 : 0;
    if (has_color) {
        if (color.size() >= sizeof(o->colors[idx])) return false;
        copy_str(o->colors[idx], sizeof(o->colors[idx]), color);
    } else {
        o->colors[idx][0] = 0;
    }
    return true;
}

}  // namespace

// ---------------------------------------------------------------- LutProviderImpl
struct omr_lut_provider {
    std::map<std::string, std::vector<uint8_t>> luts;
};

namespace {
bool ends_with_lut(const std::string& n) {
    return n.size() >= 4 && lower(n.substr(n.size() - 4)) == ".lut";
}

void scan_luts(const std::string& dir, omr_lut_provider* p, int depth) {
    if (depth > 32) return;
    DIR* d = opendir(dir.c_str());
    if (!d) return;
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
        const std::string n = e->d_name;
        if (n != "." && n != "..") names.push_back(n);
    }
    closedir(d);
    std::sort(names.begin(), names.end());   // deterministic: later basenames overwrite (HashMap.put)
    for (const auto& n : names) {
        const std::string path = dir + "/" + n;
        struct stat st;
        if (stat(path.c_str(), &st) != 0) continue;
        if (S_ISDIR(st.st_mode)) { scan_luts(path, p, depth + 1); continue; }
        if (!S_ISREG(st.st_mode) || !ends_with_lut(n) || st.st_size > (1 << 20)) continue;
        FILE* f = std::fopen(path.c_str(), "rb");
        if (!f) continue;
        std::vector<uint8_t> data((size_t)st.st_size);
        const size_t got = data.empty() ? 0 : std::fread(data.data(), 1, data.size(), f);
        std::fclose(f);
        std::vector<uint8_t> table(768);
        // "Cannot read lookup table" is logged and the file skipped (LutProviderImpl.java:52-55)
        if (got == data.size() && omr_parse_lut(data.data(), data.size(), table.data()) == OMR_OK)
            p->luts[n] = table;
    }
}
}  // namespace

extern "C" {

omr_status omr_lut_provider_create(const char* root, omr_lut_provider** out) {
    if (!out) return OMR_INVALID_ARGUMENT;
    auto* p = new omr_lut_provider();
    if (root) scan_luts(root, p, 0);
    *out = p;
    return OMR_OK;
}

void omr_lut_provider_destroy(omr_lut_provider* p) { delete p; }

int32_t omr_lut_provider_count(const omr_lut_provider* p) { return p ? (int32_t)p->luts.size() : 0; }

omr_status omr_lut_provider_add(omr_lut_provider* p, const char* name, const uint8_t lut_rgb768[768]) {
    if (!p || !name || !lut_rgb768) return OMR_INVALID_ARGUMENT;
    p->luts[name] = std::vector<uint8_t>(lut_rgb768, lut_rgb768 + 768);
    return OMR_OK;
}

const uint8_t* omr_lut_provider_get(const omr_lut_provider* p, const char* name) {
    if (!p || !name) return nullptr;
    auto it = p->luts.find(name);
    return it == p->luts.end() ? nullptr : it->second.data();
}

// ImageRegionCtx.assignParams (ImageRegionCtx.java:127-153).
omr_status omr_image_region_ctx_parse(const char* const* names, const char* const* values, int32_t n,
                                      omr_image_region_ctx* o, char* err, size_t err_cap) {
    if (!o || n < 0 || (n > 0 && (!names || !values))) return OMR_INVALID_ARGUMENT;
    std::memset(o, 0, sizeof(*o));
    MultiMap p;
    for (int32_t i = 0; i < n; ++i) {
        if (!names[i] || !values[i]) continue;
        p.entries.emplace_back(names[i], values[i]);
    }
    auto bad = [&](const std::string& msg) {
        set_err(err, err_cap, msg);
        return (omr_status)OMR_INVALID_ARGUMENT;
    };
    auto checked = [&](const char* key, const std::string** v) -> bool {
        *v = p.get(key);
        return *v != nullptr;
    };
    const std::string* v;
    // getImageIdFromString / getIntegerFromString (:187-225)
    if (!checked("imageId", &v)) return bad("Missing parameter 'imageId'");
    int64_t id;
    if (!jparse_long(*v, INT64_MIN, INT64_MAX, id)) return bad("Incorrect format for imageid parameter '" + *v + "'");
    o->image_id = id;
    if (!checked("theZ", &v)) return bad("Missing parameter 'theZ'");
    if (!jparse_int(*v, o->z)) return bad("Incorrect format for parameter value '" + *v + "'");
    if (!checked("theT", &v)) return bad("Missing parameter 'theT'");
    if (!jparse_int(*v, o->t)) return bad("Incorrect format for parameter value '" + *v + "'");
    // getTileFromString (:232-245): NumberFormatException is an IllegalArgumentException;
    // a short array throws ArrayIndexOutOfBounds (not caught -> 500).
    if ((v = p.get("tile"))) {
        const std::vector<std::string> ta = jsplit(*v, ',', -1);
        // ta[1] is parsed before ta[2] is indexed: "a,b" is a NumberFormatException (400)
        int32_t probe;
        if (ta.size() == 2 && !jparse_int(ta[1], probe)) return bad("For input string in tile '" + *v + "'");
        if (ta.size() < 3) {
            set_err(err, err_cap, "ArrayIndexOutOfBoundsException in tile '" + *v + "'");
            return OMR_INTERNAL;
        }
        o->has_tile = 1;
        // evaluation order of :238-244: x, y, (w, h), resolution
        if (!jparse_int(ta[1], o->tile.x) || !jparse_int(ta[2], o->tile.y)) return bad("For input string in tile '" + *v + "'");
        if (ta.size() == 5 && (!jparse_int(ta[3], o->tile.width) || !jparse_int(ta[4], o->tile.height)))
            return bad("For input string in tile '" + *v + "'");
        if (!jparse_int(ta[0], o->resolution)) return bad("For input string in tile '" + *v + "'");
        o->has_resolution = 1;
    }
    // getRegionFromString (:252-273)
    if ((v = p.get("region"))) {
        const std::vector<std::string> rs = jsplit(*v, ',', -1);
        if (rs.size() != 4) return bad("Region string format incorrect. Should be 'x,y,w,h'");
        if (!jparse_int(rs[0], o->region.x) || !jparse_int(rs[1], o->region.y) ||
            !jparse_int(rs[2], o->region.width) || !jparse_int(rs[3], o->region.height))
            return bad("Improper number formatting in region string " + *v);
        o->has_region = 1;
    }
    // getChannelInfoFromString (:281-326)
    o->n_channels = -1;
    if ((v = p.get("c"))) {
        const std::vector<std::string> ca = jsplit(*v, ',', -1);
        if ((int)ca.size() > OMR_MAX_REQUEST_CHANNELS) return bad("Too many channels in 'c'");
        for (size_t k = 0; k < ca.size(); ++k)
            if (!parse_channel(ca[k], o, (int)k)) return bad("Failed to parse channel '" + ca[k] + "'");
        o->n_channels = (int32_t)ca.size();
    }
    // getColorModelFromString (:333-341)
    o->model = -1;
    if ((v = p.get("m"))) {
        if (*v == "g") o->model = OMR_MODEL_GREYSCALE;
        else if (*v == "c") o->model = OMR_MODEL_RGB;
    }
    // getCompressionQualityFromString (:347-349)
    if ((v = p.get("q"))) {
        if (!jparse_float(*v, o->quality)) return bad("For input string: \"" + *v + "\"");
        o->has_quality = 1;
    }
    // getInvertedAxisFromString (:355-357): parsed, unused by the handler
    o->inverted_axis = -1;
    if ((v = p.get("ia"))) o->inverted_axis = iequals(*v, "true") ? 1 : 0;
    // getProjectionFromString (:370-402)
    o->projection = -1;
    if ((v = p.get("p"))) {
        std::vector<std::string> parts = jsplit(*v, '|', -1);
        if (parts[0] == "intmax") o->projection = OMR_PROJECTION_MAX;
        else if (parts[0] == "intmean") o->projection = OMR_PROJECTION_MEAN;
        else if (parts[0] == "intsum") o->projection = OMR_PROJECTION_SUM;
        if (parts.size() == 2) {
            const std::vector<std::string> se = jsplit(parts[1], ':', 0);
            int32_t s, e;
            // projectionStart is assigned before projectionEnd is parsed (:397-398)
            if (!se.empty() && jparse_int(se[0], s)) {
                o->has_projection_start = 1;
                o->projection_start = s;
                if (se.size() < 2) {           // ArrayIndexOutOfBounds is not caught (:399)
                    set_err(err, err_cap, "ArrayIndexOutOfBoundsException in p '" + *v + "'");
                    return OMR_INTERNAL;
                }
                if (jparse_int(se[1], e)) { o->has_projection_end = 1; o->projection_end = e; }
            } else if (se.empty()) {
                set_err(err, err_cap, "ArrayIndexOutOfBoundsException in p '" + *v + "'");
                return OMR_INTERNAL;
            }
        }
    }
    // maps (:138,143-145): Json.decodeValue(maps, List.class); DecodeException is not an IAE
    o->n_maps = -1;
    if ((v = p.get("maps"))) {
        JsonCursor jc(*v);
        jc.ws();
        bool ok = jc.i < v->size() && (*v)[jc.i] == '[';
        int count = 0;
        if (ok) {
            ++jc.i;
            jc.ws();
            if (jc.i < v->size() && (*v)[jc.i] == ']') {
                ++jc.i;
            } else {
                for (;;) {
                    int kind, rev = OMR_MAP_NONE;
                    if (!jc.value(&kind, 1, &rev)) { ok = false; break; }
                    if (count < OMR_MAX_REQUEST_CHANNELS)
                        o->map_reverse[count] = kind == 0 ? OMR_MAP_NULL : kind == 3 ? rev : OMR_MAP_BAD;
                    ++count;
                    jc.ws();
                    if (jc.i < v->size() && (*v)[jc.i] == ',') { ++jc.i; continue; }
                    if (jc.i < v->size() && (*v)[jc.i] == ']') { ++jc.i; break; }
                    ok = false;
                    break;
                }
            }
            // Jackson 2.x ignores trailing tokens after the root value (FAIL_ON_TRAILING_TOKENS off)
        }
        if (!ok) {
            set_err(err, err_cap, "Failed to decode maps: " + *v);
            return OMR_INTERNAL;
        }
        o->n_maps = std::min(count, (int)OMR_MAX_REQUEST_CHANNELS);
    }
    // flip (:139-142)
    if ((v = p.get("flip"))) {
        const std::string f = lower(*v);
        o->flip_h = f.find('h') != std::string::npos;
        o->flip_v = f.find('v') != std::string::npos;
    }
    // format (:146)
    v = p.get("format");
    const std::string fmt = v ? *v : "jpeg";
    if (fmt.size() >= sizeof(o->format)) copy_str(o->format, sizeof(o->format), "?");
    else copy_str(o->format, sizeof(o->format), fmt);
    // createCacheKey (:165-177): sorted names, "<class>:key=value..." UTF-8, sipHash24 default key
    std::vector<std::string> keys = p.names();
    std::sort(keys.begin(), keys.end());
    std::string sb = "com.glencoesoftware.omero.ms.image.region.ImageRegionCtx";
    for (const auto& k : keys) sb += ":" + k + "=" + *p.get(k.c_str());
    hash_hex(siphash24(reinterpret_cast<const uint8_t*>(sb.data()), sb.size(), 0x0706050403020100ull,
                       0x0f0e0d0c0b0a0908ull),
             o->cache_key);
    set_err(err, err_cap, "");
    return OMR_OK;
}

// ShapeMaskCtx(MultiMap, String) (ShapeMaskCtx.java:61-72) + cacheKey (:77-81).
omr_status omr_shape_mask_ctx_parse(const char* const* names, const char* const* values, int32_t n,
                                    omr_shape_mask_ctx* o, char* err, size_t err_cap) {
    if (!o || n < 0 || (n > 0 && (!names || !values))) return OMR_INVALID_ARGUMENT;
    std::memset(o, 0, sizeof(*o));
    MultiMap p;
    for (int32_t i = 0; i < n; ++i)
        if (names[i] && values[i]) p.entries.emplace_back(names[i], values[i]);
    const std::string* v = p.get("shapeId");
    int64_t id;
    // Long.parseLong(null) and bad digits throw NumberFormatException; the verticle does not
    // catch it (ImageRegionMicroserviceVerticle.java:365-366), so it is a 500.
    if (!v || !jparse_long(*v, INT64_MIN, INT64_MAX, id)) {
        set_err(err, err_cap, std::string("NumberFormatException: shapeId '") + (v ? *v : "null") + "'");
        return OMR_INTERNAL;
    }
    o->shape_id = id;
    v = p.get("color");
    o->has_color = v != nullptr;
    if (v) {
        if (v->size() >= sizeof(o->color)) {
            set_err(err, err_cap, "color too long");
            return OMR_INVALID_ARGUMENT;
        }
        copy_str(o->color, sizeof(o->color), *v);
    }
    if ((v = p.get("flip"))) {
        const std::string f = lower(*v);
        o->flip_h = f.find('h') != std::string::npos;
        o->flip_v = f.find('v') != std::string::npos;
    }
    const std::string key = "ome.model.roi.Mask:" + std::to_string(id) + ":" + (o->has_color ? o->color : "null");
    copy_str(o->cache_key, sizeof(o->cache_key), key);
    set_err(err, err_cap, "");
    return OMR_OK;
}

// ImageRegionRequestHandler.createRenderingDef (:258-300) as the Renderer sees it: QuantumDef
// 0/255/255, greyscale model, per channel linear k=1 no NR, window = type range, red, active c<3.
omr_status omr_create_rendering_def(int32_t pixel_type, int32_t size_c, omr_quantum_def* qdef,
                                    omr_channel_binding* channels) {
    if (!qdef || !channels || size_c < 0) return OMR_INVALID_ARGUMENT;
    double lo, hi;
    switch (pixel_type) {   // StatsFactory.initPixelsRange
        case OMR_PIXELS_INT8: lo = -128.0; hi = 127.0; break;
        case OMR_PIXELS_UINT8: lo = 0.0; hi = 255.0; break;
        case OMR_PIXELS_INT16: lo = -32768.0; hi = 32767.0; break;
        case OMR_PIXELS_UINT16: lo = 0.0; hi = 65535.0; break;
        case OMR_PIXELS_INT32: lo = -2147483648.0; hi = 2147483647.0; break;
        case OMR_PIXELS_UINT32: lo = 0.0; hi = 4294967295.0; break;
        case OMR_PIXELS_FLOAT:
        case OMR_PIXELS_DOUBLE: lo = 0.0; hi = 1.0; break;
        default: return OMR_INVALID_ARGUMENT;
    }
    qdef->cd_start = 0;
    qdef->cd_end = 255;
    qdef->bit_resolution = 255;
    qdef->model = OMR_MODEL_GREYSCALE;
    for (int32_t c = 0; c < size_c; ++c) {
        omr_channel_binding& b = channels[c];
        std::memset(&b, 0, sizeof(b));
        b.active = c < 3;
        b.family = OMR_FAMILY_LINEAR;
        b.coefficient = 1.0;
        b.noise_reduction = 0;
        b.reverse = 0;
        b.input_start = lo;
        b.input_end = hi;
        b.global_min = lo;
        b.global_max = hi;
        b.rgba[0] = 255; b.rgba[1] = 0; b.rgba[2] = 0; b.rgba[3] = 255;
        b.lut = nullptr;
    }
    return OMR_OK;
}

// ImageRegionRequestHandler.updateSettings (:689-741).  Windows and colours are indexed by the
// channel index c (idx advances for every channel, active or not, :733), maps likewise (:716).
omr_status omr_update_settings(const omr_image_region_ctx* rc, int32_t size_c, omr_quantum_def* qdef,
                               omr_channel_binding* channels, const omr_lut_provider* luts,
                               char* err, size_t err_cap) {
    if (!rc || !qdef || !channels || size_c < 0) return OMR_INVALID_ARGUMENT;
    auto npe = [&](const std::string& what) {
        set_err(err, err_cap, what);
        return (omr_status)OMR_INTERNAL;
    };
    if (rc->n_channels < 0) return npe("NullPointerException: channels is null (no 'c' parameter)");
    for (int32_t c = 0; c < size_c; ++c) {
        bool active = false;
        for (int32_t k = 0; k < rc->n_channels; ++k) active = active || rc->channels[k] == c + 1;
        omr_channel_binding& b = channels[c];
        b.active = active;
        if (!active) continue;
        const int idx = c;
        if (idx >= rc->n_channels) return npe("IndexOutOfBoundsException: windows.get(" + std::to_string(idx) + ")");
        if (!rc->window_set[idx]) return npe("NullPointerException: channel window is null");
        b.input_start = (double)rc->windows[idx][0];
        b.input_end = (double)rc->windows[idx][1];
        if (!rc->color_set[idx]) return npe("NullPointerException: channel colour is null");
        const std::string color = rc->colors[idx];
        if (color.size() >= 4 && color.compare(color.size() - 4, 4, ".lut") == 0) {
            // setChannelLookupTable: the reader is resolved by name at render time; a missing
            // one leaves the channel on its colour (LutProviderImpl.getLutReaders -> null).
            b.lut = luts ? omr_lut_provider_get(luts, color.c_str()) : nullptr;
        } else {
            int32_t rgba[4];
            if (omr_split_html_color(color.c_str(), rgba) != OMR_OK)
                return npe("NullPointerException: splitHTMLColor('" + color + "') returned null");
            for (int i = 0; i < 4; ++i)
                if (rgba[i] < 0 || rgba[i] > 255) return npe("colour component out of range in '" + color + "'");
            for (int i = 0; i < 4; ++i) b.rgba[i] = (uint8_t)rgba[i];
            b.lut = nullptr;
        }
        if (rc->n_maps >= 0 && c < rc->n_maps) {
            const int32_t m = rc->map_reverse[c];
            if (m == OMR_MAP_BAD) return npe("ClassCastException: maps[" + std::to_string(c) + "]");
            if (m == OMR_MAP_REVERSE) b.reverse = 1;
        }
    }
    if (rc->model < 0) return npe("NullPointerException: colour model 'm' is null");
    qdef->model = rc->model;
    set_err(err, err_cap, "");
    return OMR_OK;
}

}  // extern "C"
