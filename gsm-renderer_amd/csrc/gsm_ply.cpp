// gsm_ply.cpp -- PLY ingestion for the GlobalRenderer input (include/gsm_ply.h).
//
// A host-side restatement of the reference's PLYLoader (Sources/Renderer/Utils/PLYLoader.swift)
// and GaussianSceneBuilder (Sources/Renderer/Utils/Scene.swift).  Every function cites the
// Swift lines it follows.  Deliberate differences, all documented in DESIGN.md:
//   * Swift's Array.sort is not stable; the SH-property sort and the Morton sort here are
//     (ties keep file order), so equal keys give one defined order;
//   * out-of-range chunk indices of an inconsistent compressed file are an error here instead
//     of an out-of-bounds read;
//   * an element count above UInt32.max is an invalid header line instead of a trap.
// Float arithmetic is single precision with the reference's operation order; exp, sqrt and
// quaternion normalisation use the C library (results within a few ulp of Apple's simd/libm).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gsm_ply.h"
#include "gsm_types.h"

struct gsm_ply_scene {
    std::vector<float> pos, scale, rot, opacity;  // [n][3], [n][3], [n][4] (x, y, z, w), [n]
    std::vector<float> harmonics;                 // dataset.harmonics (planar per gaussian)
    uint32_t n = 0, shComponents = 0;
    int compressed = 0;
};

namespace {

thread_local std::string g_lastError;

gsm_ply_status fail(gsm_ply_status s, const std::string& msg) {
    g_lastError = msg;
    return s;
}

// ---------------------------------------------------------------------------------------
// PLYHeader (PLYLoader.swift:6-90, 115-218)
// ---------------------------------------------------------------------------------------
enum class PType { I8, U8, I16, U16, I32, U32, F32, F64 };

int width(PType t) {  // PrimitivePropertyType.byteWidth (:57-63)
    switch (t) {
        case PType::I8: case PType::U8: return 1;
        case PType::I16: case PType::U16: return 2;
        case PType::I32: case PType::U32: case PType::F32: return 4;
        case PType::F64: return 8;
    }
    return 0;
}

bool type_from_string(const std::string& s, PType* t) {  // fromString (:203-214)
    if (s == "int8" || s == "char") *t = PType::I8;
    else if (s == "uint8" || s == "uchar") *t = PType::U8;
    else if (s == "int16" || s == "short") *t = PType::I16;
    else if (s == "uint16" || s == "ushort") *t = PType::U16;
    else if (s == "int32" || s == "int") *t = PType::I32;
    else if (s == "uint32" || s == "uint") *t = PType::U32;
    else if (s == "float32" || s == "float") *t = PType::F32;
    else if (s == "float64" || s == "double") *t = PType::F64;
    else return false;
    return true;
}

struct Property {
    std::string name;
    bool list = false;
    PType type = PType::F32;  // value type (primitive) or list value type
    int byteWidth() const { return list ? 0 : width(type); }  // (:39-44)
};
struct Element {
    std::string name;
    uint32_t count = 0;
    std::vector<Property> props;
};
enum class Format { Ascii, BinaryLE, BinaryBE };
struct Header {
    Format format = Format::BinaryLE;
    std::vector<Element> elements;
};

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\v' || c == '\f'; }
bool is_word(char c) { return std::isalnum((unsigned char)c) || c == '_'; }

// Tokenise a header line by the grammar of the reference's regexes (whole-line matches):
// leading whitespace, then tokens separated by runs of whitespace, nothing after the last.
// Returns false when the line ends in whitespace or a token breaks `classes` (w = \w+,
// S = \S+, d = \d+).
bool match_tokens(const std::string& line, const char* classes, std::vector<std::string>* out) {
    out->clear();
    size_t i = 0;
    while (i < line.size() && is_ws(line[i])) i++;
    for (size_t k = 0; classes[k]; ++k) {
        if (k > 0) {  // \s+ between tokens
            size_t j = i;
            while (j < line.size() && is_ws(line[j])) j++;
            if (j == i) return false;
            i = j;
        }
        size_t j = i;
        while (j < line.size() && !is_ws(line[j])) j++;
        if (j == i) return false;
        const std::string tok = line.substr(i, j - i);
        for (char c : tok) {
            if (classes[k] == 'w' && !is_word(c)) return false;
            if (classes[k] == 'd' && !std::isdigit((unsigned char)c)) return false;
        }
        out->push_back(tok);
        i = j;
    }
    return i == line.size();
}

// PLYHeader.decodeASCII (PLYLoader.swift:115-201)
gsm_ply_status decode_header(const std::string& text, Header* h) {
    for (unsigned char c : text)
        if (c >= 0x80) return fail(GSM_PLY_ERR_HEADER_INVALID_CHARACTERS, "Invalid characters in header");
    bool haveFormat = false;
    size_t p = 0;
    while (p < text.size()) {  // enumerateLines: \n, \r\n and \r end a line
        size_t e = p;
        while (e < text.size() && text[e] != '\n' && text[e] != '\r') e++;
        const std::string line = text.substr(p, e - p);
        if (e + 1 < text.size() && text[e] == '\r' && text[e + 1] == '\n') p = e + 2;
        else p = e < text.size() ? e + 1 : e;
        // first whitespace-separated component
        size_t a = 0;
        while (a < line.size() && is_ws(line[a])) a++;
        if (a == line.size()) continue;
        size_t b = a;
        while (b < line.size() && !is_ws(line[b])) b++;
        const std::string kw = line.substr(a, b - a);
        std::vector<std::string> t;
        if (kw == "ply" || kw == "comment" || kw == "obj_info") continue;
        if (kw == "format") {
            if (haveFormat) return fail(GSM_PLY_ERR_HEADER_UNEXPECTED_KEYWORD, "Unexpected keyword: \"format\"");
            if (!match_tokens(line, "SwS", &t) || t[0] != "format")
                return fail(GSM_PLY_ERR_HEADER_INVALID_LINE, "Invalid line: \"" + line + "\"");
            if (t[1] == "ascii") h->format = Format::Ascii;
            else if (t[1] == "binary_little_endian") h->format = Format::BinaryLE;
            else if (t[1] == "binary_big_endian") h->format = Format::BinaryBE;
            else return fail(GSM_PLY_ERR_HEADER_INVALID_FORMAT_TYPE, "Invalid format type: " + t[1]);
            haveFormat = true;
        } else if (kw == "element") {
            if (!haveFormat) return fail(GSM_PLY_ERR_HEADER_UNEXPECTED_KEYWORD, "Unexpected keyword: \"element\"");
            if (!match_tokens(line, "SSd", &t) || t[0] != "element")
                return fail(GSM_PLY_ERR_HEADER_INVALID_LINE, "Invalid line: \"" + line + "\"");
            unsigned long long c = 0;
            for (char d : t[2]) {
                c = c * 10 + (unsigned)(d - '0');
                if (c > 0xFFFFFFFFull) return fail(GSM_PLY_ERR_HEADER_INVALID_LINE, "Invalid line: \"" + line + "\"");
            }
            Element el;
            el.name = t[1];
            el.count = (uint32_t)c;
            h->elements.push_back(el);
        } else if (kw == "property") {
            if (!haveFormat || h->elements.empty())
                return fail(GSM_PLY_ERR_HEADER_UNEXPECTED_KEYWORD, "Unexpected keyword: \"property\"");
            Property pr;
            if (match_tokens(line, "SSwwS", &t) && t[0] == "property" && t[1] == "list") {
                PType ct, vt;
                if (!type_from_string(t[2], &ct)) return fail(GSM_PLY_ERR_HEADER_UNKNOWN_PROPERTY_TYPE, "Unknown property type: " + t[2]);
                if (!type_from_string(t[3], &vt)) return fail(GSM_PLY_ERR_HEADER_UNKNOWN_PROPERTY_TYPE, "Unknown property type: " + t[3]);
                pr.name = t[4];
                pr.list = true;
                pr.type = vt;
            } else if (match_tokens(line, "SwS", &t) && t[0] == "property") {
                PType vt;
                if (!type_from_string(t[1], &vt)) return fail(GSM_PLY_ERR_HEADER_UNKNOWN_PROPERTY_TYPE, "Unknown property type: " + t[1]);
                pr.name = t[2];
                pr.type = vt;
            } else {
                return fail(GSM_PLY_ERR_HEADER_INVALID_LINE, "Invalid line: \"" + line + "\"");
            }
            h->elements.back().props.push_back(pr);
        } else if (kw == "end_header") {
            break;
        } else {
            return fail(GSM_PLY_ERR_HEADER_UNKNOWN_KEYWORD, "Unknown keyword: \"" + kw + "\"");
        }
    }
    if (!haveFormat) return fail(GSM_PLY_ERR_HEADER_FORMAT_MISSING, "Header format missing");
    return GSM_PLY_OK;
}

// ---------------------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------------------
template <class T>
T load_le(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    return v;
}

float prop_float(const uint8_t* p, PType t) {  // getFloat (PLYLoader.swift:598-616)
    switch (t) {
        case PType::F32: return load_le<float>(p);
        case PType::F64: return (float)load_le<double>(p);
        case PType::U8: return (float)load_le<uint8_t>(p) / 255.0f;
        case PType::I8: return (float)load_le<int8_t>(p);
        case PType::I16: return (float)load_le<int16_t>(p);
        case PType::U16: return (float)load_le<uint16_t>(p);
        case PType::I32: return (float)load_le<int32_t>(p);
        case PType::U32: return (float)load_le<uint32_t>(p);
    }
    return 0.0f;
}

template <class F>
void parallel_for(size_t n, F&& f) {
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 65536) nt = 1;
    const size_t per = (n + nt - 1) / nt;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) {
        const size_t b = per * t, e = std::min(n, b + per);
        if (b < e) th.emplace_back([&f, b, e] { f(b, e); });
    }
    f(0, std::min(n, per));
    for (auto& x : th) x.join();
}

// GaussianSceneBuilder.bounds(of:) centre (Scene.swift:172-187), then the recentering of
// PLYLoader.swift:497-504 / 723-731
void recenter(gsm_ply_scene* s) {
    if (s->n == 0) return;
    float mn[3] = {s->pos[0], s->pos[1], s->pos[2]}, mx[3] = {s->pos[0], s->pos[1], s->pos[2]};
    for (uint32_t i = 0; i < s->n; ++i)
        for (int c = 0; c < 3; ++c) {
            mn[c] = std::min(mn[c], s->pos[3 * i + c]);
            mx[c] = std::max(mx[c], s->pos[3 * i + c]);
        }
    float ctr[3];
    for (int c = 0; c < 3; ++c) ctr[c] = (mn[c] + mx[c]) * 0.5f;
    const float len = std::sqrt((ctr[0] * ctr[0] + ctr[1] * ctr[1]) + ctr[2] * ctr[2]);
    if (len > 1e-6f)
        for (uint32_t i = 0; i < s->n; ++i)
            for (int c = 0; c < 3; ++c) s->pos[3 * i + c] -= ctr[c];
}

void alloc_records(gsm_ply_scene* s, size_t n) {
    s->n = (uint32_t)n;
    s->pos.assign(3 * n, 0.0f);
    s->scale.assign(3 * n, 0.0f);
    s->rot.assign(4 * n, 0.0f);
    s->opacity.assign(n, 0.0f);
}

// ---------------------------------------------------------------------------------------
// loadCompressed (PLYLoader.swift:291-514)
// ---------------------------------------------------------------------------------------
gsm_ply_status load_compressed(const uint8_t* data, size_t size, const Header& h, size_t bodyStart,
                               gsm_ply_scene* s) {
    const Element* chunk = nullptr;
    const Element* vertex = nullptr;
    const Element* sh = nullptr;
    for (const auto& e : h.elements) {
        if (!chunk && e.name == "chunk") chunk = &e;
        if (!vertex && e.name == "vertex") vertex = &e;
        if (!sh && e.name == "sh") sh = &e;
    }
    if (!chunk || !vertex) return fail(GSM_PLY_ERR_MISSING_CHUNK_ELEMENT, "Missing chunk element in compressed PLY");
    const size_t chunkCount = chunk->count, vertexCount = vertex->count;
    auto offsets = [](const Element& e, size_t* stride) {
        std::vector<std::pair<std::string, size_t>> o;
        size_t st = 0;
        for (const auto& p : e.props) {
            o.emplace_back(p.name, st);
            st += (size_t)p.byteWidth();
        }
        *stride = st;
        return o;
    };
    size_t chunkStride, vertexStride, shStride = 0;
    const auto chunkOff = offsets(*chunk, &chunkStride);
    const auto vertexOff = offsets(*vertex, &vertexStride);
    if (sh) offsets(*sh, &shStride);
    const size_t chunkDataStart = bodyStart;
    const size_t vertexDataStart = chunkDataStart + chunkStride * chunkCount;
    const size_t shDataStart = vertexDataStart + vertexStride * vertexCount;
    if (size < shDataStart + shStride * vertexCount) return fail(GSM_PLY_ERR_INSUFFICIENT_DATA, "Insufficient data in PLY file");
    if (vertexCount > 0 && (vertexCount - 1) / 256 >= chunkCount)
        return fail(GSM_PLY_ERR_INSUFFICIENT_DATA, "Insufficient data in PLY file (chunks for every 256 vertices)");
    auto find = [](const std::vector<std::pair<std::string, size_t>>& o, const char* name) -> long {
        for (const auto& p : o)
            if (p.first == name) return (long)p.second;
        return -1;
    };
    static const char* kChunk[18] = {"min_x", "min_y", "min_z", "max_x", "max_y", "max_z",
                                     "min_scale_x", "min_scale_y", "min_scale_z", "max_scale_x", "max_scale_y", "max_scale_z",
                                     "min_r", "min_g", "min_b", "max_r", "max_g", "max_b"};
    long co[18];
    for (int k = 0; k < 18; ++k) co[k] = find(chunkOff, kChunk[k]);
    const long oPos = find(vertexOff, "packed_position"), oRot = find(vertexOff, "packed_rotation");
    const long oScale = find(vertexOff, "packed_scale"), oColor = find(vertexOff, "packed_color");
    // The reader takes 4 bytes at every one of these offsets whatever the declared type (as the
    // reference's loadUnaligned, PLYLoader.swift:318-334).  A narrower property placed last in its
    // element would make that read run past the element -- and, for the last chunk or vertex,
    // past the buffer: such files are rejected instead.
    for (int k = 0; k < 18; ++k)
        if (co[k] >= 0 && (size_t)co[k] + 4 > chunkStride)
            return fail(GSM_PLY_ERR_INSUFFICIENT_DATA, "Compressed PLY chunk property narrower than 4 bytes at the end of the element");
    for (long o : {oPos, oRot, oScale, oColor})
        if (o >= 0 && (size_t)o + 4 > vertexStride)
            return fail(GSM_PLY_ERR_INSUFFICIENT_DATA, "Compressed PLY packed property narrower than 4 bytes at the end of the element");

    alloc_records(s, vertexCount);
    s->harmonics.assign(3 * vertexCount, 0.0f);
    auto unorm = [](uint32_t v, int bits) {  // unpackUnorm (:355-358)
        const uint32_t mask = (1u << bits) - 1u;
        return (float)(v & mask) / (float)mask;
    };
    auto lerp = [](float a, float b, float t) { return a * (1.0f - t) + b * t; };  // (:400-402)
    const float SH_C0 = 0.28209479177387814f;
    const float norm = 1.0f / (std::sqrt(2.0f) * 0.5f);
    parallel_for(vertexCount, [&](size_t b, size_t e) {
        for (size_t v = b; v < e; ++v) {
            const uint8_t* cp = data + chunkDataStart + (v / 256) * chunkStride;
            float c[18];
            for (int k = 0; k < 18; ++k) c[k] = co[k] < 0 ? 0.0f : load_le<float>(cp + co[k]);  // getChunkFloat
            const uint8_t* vp = data + vertexDataStart + v * vertexStride;
            auto u32 = [&](long o) { return o < 0 ? 0u : load_le<uint32_t>(vp + o); };  // getVertexUInt32
            const uint32_t pp = u32(oPos), pr = u32(oRot), ps = u32(oScale), pc = u32(oColor);
            // unpack111011 (:360-365) position
            const float px = unorm(pp >> 21, 11), py = unorm(pp >> 11, 10), pz = unorm(pp, 11);
            s->pos[3 * v + 0] = lerp(c[0], c[3], px);
            s->pos[3 * v + 1] = lerp(c[1], c[4], py);
            s->pos[3 * v + 2] = lerp(c[2], c[5], pz);
            // unpackRotation (:375-398): (x, y, z, w) of the simd_quatf
            const float a = (unorm(pr >> 20, 10) - 0.5f) * norm;
            const float bb = (unorm(pr >> 10, 10) - 0.5f) * norm;
            const float cc = (unorm(pr, 10) - 0.5f) * norm;
            const float m = std::sqrt(std::max(0.0f, 1.0f - ((a * a + bb * bb) + cc * cc)));
            float q[4];
            switch (pr >> 30) {
                case 0: q[0] = a; q[1] = bb; q[2] = cc; q[3] = m; break;
                case 1: q[0] = m; q[1] = bb; q[2] = cc; q[3] = a; break;
                case 2: q[0] = bb; q[1] = m; q[2] = cc; q[3] = a; break;
                default: q[0] = bb; q[1] = cc; q[2] = m; q[3] = a; break;
            }
            std::memcpy(&s->rot[4 * v], q, sizeof(q));
            // scale: exp of the interpolated log scale (:449-454)
            const float sx = unorm(ps >> 21, 11), sy = unorm(ps >> 11, 10), sz = unorm(ps, 11);
            s->scale[3 * v + 0] = std::exp(lerp(c[6], c[9], sx));
            s->scale[3 * v + 1] = std::exp(lerp(c[7], c[10], sy));
            s->scale[3 * v + 2] = std::exp(lerp(c[8], c[11], sz));
            // unpack8888 (:367-373): colour -> SH DC, opacity (:456-468)
            const float cr = unorm(pc >> 24, 8), cg = unorm(pc >> 16, 8), cb = unorm(pc >> 8, 8), cw = unorm(pc, 8);
            s->opacity[v] = cw;
            s->harmonics[3 * v + 0] = (lerp(c[12], c[15], cr) - 0.5f) / SH_C0;
            s->harmonics[3 * v + 1] = (lerp(c[13], c[16], cg) - 0.5f) / SH_C0;
            s->harmonics[3 * v + 2] = (lerp(c[14], c[17], cb) - 0.5f) / SH_C0;
        }
    });
    s->shComponents = 1;
    s->compressed = 1;
    recenter(s);
    return GSM_PLY_OK;
}

// ---------------------------------------------------------------------------------------
// loadStandard (PLYLoader.swift:518-741)
// ---------------------------------------------------------------------------------------
int sh_sort_key(const std::string& name) {  // shSortKey (:576-581); Int.max for other names
    auto num = [](const std::string& s) {
        if (s.empty()) return 0;
        long v = 0;
        for (char c : s) {
            if (!std::isdigit((unsigned char)c)) return 0;  // Int(...) ?? 0
            v = v * 10 + (c - '0');
            if (v > 1000000000) return 0;
        }
        return (int)v;
    };
    if (name.rfind("f_dc_", 0) == 0) return num(name.substr(5));
    if (name.rfind("f_rest_", 0) == 0) return 3 + num(name.substr(7));
    if (name.rfind("sh_", 0) == 0) return num(name.substr(3));
    return 0x7FFFFFFF;
}

gsm_ply_status load_standard(const uint8_t* data, size_t size, const Element& vertex, size_t bodyStart,
                             gsm_ply_scene* s) {
    for (const auto& p : vertex.props)
        if (p.list) return fail(GSM_PLY_ERR_LIST_PROPERTIES_NOT_SUPPORTED, "List properties are not supported");
    const size_t vertexCount = vertex.count;
    std::vector<size_t> off;
    size_t stride = 0;
    for (const auto& p : vertex.props) {
        off.push_back(stride);
        stride += (size_t)p.byteWidth();
    }
    if (size - bodyStart < stride * vertexCount) return fail(GSM_PLY_ERR_INSUFFICIENT_DATA, "Insufficient data in PLY file");
    int ix = -1, iy = -1, iz = -1, is0 = -1, is1 = -1, is2 = -1, ir0 = -1, ir1 = -1, ir2 = -1, ir3 = -1, iop = -1;
    std::vector<std::pair<std::string, int>> shMap;
    for (size_t i = 0; i < vertex.props.size(); ++i) {
        std::string n = vertex.props[i].name;
        for (auto& c : n) c = (char)std::tolower((unsigned char)c);
        const int k = (int)i;
        if (n == "x" || n == "px" || n == "pos_x" || n == "position_x") ix = k;
        else if (n == "y" || n == "py" || n == "pos_y" || n == "position_y") iy = k;
        else if (n == "z" || n == "pz" || n == "pos_z" || n == "position_z") iz = k;
        else if (n == "scale_0" || n == "scale0" || n == "sx" || n == "scale_x") is0 = k;
        else if (n == "scale_1" || n == "scale1" || n == "sy" || n == "scale_y") is1 = k;
        else if (n == "scale_2" || n == "scale2" || n == "sz" || n == "scale_z") is2 = k;
        else if (n == "rot_0" || n == "rot0" || n == "qw" || n == "rotation_w") ir0 = k;
        else if (n == "rot_1" || n == "rot1" || n == "qx" || n == "rotation_x") ir1 = k;
        else if (n == "rot_2" || n == "rot2" || n == "qy" || n == "rotation_y") ir2 = k;
        else if (n == "rot_3" || n == "rot3" || n == "qz" || n == "rotation_z") ir3 = k;
        else if (n == "opacity" || n == "alpha") iop = k;
        else if (n.rfind("f_dc_", 0) == 0 || n.rfind("f_rest_", 0) == 0 || n.rfind("sh_", 0) == 0 ||
                 n.rfind("spherical_harmonics_", 0) == 0)
            shMap.emplace_back(n, k);
    }
    if (ix < 0 || iy < 0 || iz < 0)
        return fail(GSM_PLY_ERR_MISSING_REQUIRED_PROPERTIES, "Missing required properties: x, y, z");
    std::stable_sort(shMap.begin(), shMap.end(),
                     [](const auto& a, const auto& b) { return sh_sort_key(a.first) < sh_sort_key(b.first); });
    std::vector<int> idxSh;
    for (const auto& p : shMap) idxSh.push_back(p.second);
    const size_t shStride = idxSh.size();
    const uint8_t* body = data + bodyStart;
    auto get = [&](size_t v, int idx) {
        return idx < 0 ? 0.0f : prop_float(body + v * stride + off[(size_t)idx], vertex.props[(size_t)idx].type);
    };
    // format detection on the first min(100, n) vertices (:618-646)
    bool scaleIsLogSpace = true, opacityIsLogit = true;
    const size_t sampleCount = std::min<size_t>(100, vertexCount);
    std::vector<float> ss, so;
    for (size_t v = 0; v < sampleCount; ++v) {
        if (is0 >= 0) ss.push_back(get(v, is0));
        if (iop >= 0) so.push_back(get(v, iop));
    }
    if (!ss.empty()) {
        bool neg = false, large = false;
        float sum = 0.0f;
        for (float x : ss) {
            neg = neg || x < 0.0f;
            large = large || x > 1.0f;
            sum = sum + x;
        }
        const float avg = sum / (float)ss.size();
        if (neg) scaleIsLogSpace = true;
        else if (!large && avg > 0.0f && avg < 0.5f) scaleIsLogSpace = false;
    }
    if (!so.empty()) {
        float mn = so[0], mx = so[0];
        for (float x : so) {
            mn = std::min(mn, x);
            mx = std::max(mx, x);
        }
        opacityIsLogit = mn < 0.0f || mx > 1.0f;
    }
    // placeholder vertices are skipped (:655-657): keep flags, then compacted positions
    std::vector<uint32_t> keep(vertexCount);
    parallel_for(vertexCount, [&](size_t b, size_t e) {
        for (size_t v = b; v < e; ++v) {
            const float s0 = get(v, is0), s1 = get(v, is1), s2 = get(v, is2), op = get(v, iop);
            keep[v] = !(s0 == 2.0f && s1 == 2.0f && s2 == 2.0f && std::fabs(op - 4.8402f) < 0.001f);
        }
    });
    std::vector<size_t> dst(vertexCount + 1, 0);
    for (size_t v = 0; v < vertexCount; ++v) dst[v + 1] = dst[v] + keep[v];
    const size_t n = dst[vertexCount];
    alloc_records(s, n);
    std::vector<float> coeffs(n * shStride);  // PLY order per vertex
    parallel_for(vertexCount, [&](size_t b, size_t e) {
        for (size_t v = b; v < e; ++v) {
            if (!keep[v]) continue;
            const size_t o = dst[v];
            const float s0 = get(v, is0), s1 = get(v, is1), s2 = get(v, is2), opRaw = get(v, iop);
            s->pos[3 * o + 0] = get(v, ix);
            s->pos[3 * o + 1] = get(v, iy);
            s->pos[3 * o + 2] = get(v, iz);
            s->scale[3 * o + 0] = scaleIsLogSpace ? std::exp(s0) : s0;
            s->scale[3 * o + 1] = scaleIsLogSpace ? std::exp(s1) : s1;
            s->scale[3 * o + 2] = scaleIsLogSpace ? std::exp(s2) : s2;
            // simd_normalize(simd_quatf(ix: r1, iy: r2, iz: r3, r: r0)) (:668-673)
            const float q[4] = {get(v, ir1), get(v, ir2), get(v, ir3), get(v, ir0)};
            const float len = std::sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
            for (int c = 0; c < 4; ++c) s->rot[4 * o + c] = q[c] / len;
            s->opacity[o] = opacityIsLogit ? 1.0f / (1.0f + std::exp(-opRaw)) : opRaw;  // (:676)
            for (size_t k = 0; k < shStride; ++k) coeffs[o * shStride + k] = get(v, idxSh[k]);
        }
    });
    // PLY [DC_R, DC_G, DC_B, R1.., G1.., B1..] -> planar [R0.., G0.., B0..] (:687-721)
    const size_t shComponents = shStride == 0 ? 0 : shStride / 3;
    if (shComponents > 0) {
        const size_t hoc = shComponents - 1;
        s->harmonics.assign(n * shStride, 0.0f);
        for (size_t i = 0; i < n; ++i) {
            const float* src = &coeffs[i * shStride];
            float* d = &s->harmonics[i * shStride];
            d[0] = src[0];
            for (size_t c = 0; c < hoc; ++c) d[1 + c] = src[3 + c];
            d[shComponents] = src[1];
            for (size_t c = 0; c < hoc; ++c) d[shComponents + 1 + c] = src[3 + hoc + c];
            d[2 * shComponents] = src[2];
            for (size_t c = 0; c < hoc; ++c) d[2 * shComponents + 1 + c] = src[3 + 2 * hoc + c];
        }
    } else {
        s->harmonics.clear();
    }
    s->shComponents = (uint32_t)shComponents;
    s->compressed = 0;
    recenter(s);
    return GSM_PLY_OK;
}

// PLYLoader.load(url:) (PLYLoader.swift:254-287)
gsm_ply_status load_bytes(const uint8_t* data, size_t size, gsm_ply_scene** out) {
    static const char kLF[] = "end_header\n", kCRLF[] = "end_header\r\n";
    auto findSeq = [&](const char* pat) -> long {
        const size_t m = std::strlen(pat);
        if (size < m) return -1;
        const uint8_t* it = std::search(data, data + size, (const uint8_t*)pat, (const uint8_t*)pat + m);
        return it == data + size ? -1 : (long)(it - data) + (long)m;
    };
    long end = findSeq(kLF);
    if (end < 0) end = findSeq(kCRLF);
    if (end < 0) return fail(GSM_PLY_ERR_INVALID_HEADER, "Invalid PLY header");
    Header h;
    gsm_ply_status st = decode_header(std::string((const char*)data, (size_t)end), &h);
    if (st != GSM_PLY_OK) return st;
    if (h.format != Format::BinaryLE)
        return fail(GSM_PLY_ERR_UNSUPPORTED_FORMAT,
                    std::string("Unsupported PLY format: ") + (h.format == Format::Ascii ? "ascii" : "binaryBigEndian"));
    const Element* vertex = nullptr;
    bool hasChunk = false;
    for (const auto& e : h.elements) {
        if (!vertex && e.name == "vertex") vertex = &e;
        hasChunk = hasChunk || e.name == "chunk";
    }
    if (!vertex) return fail(GSM_PLY_ERR_MISSING_VERTEX_ELEMENT, "Missing vertex element");
    auto has = [&](const char* n) {
        for (const auto& p : vertex->props)
            if (p.name == n) return true;
        return false;
    };
    const bool compressed = hasChunk && has("packed_position") && has("packed_rotation") && has("packed_scale") &&
                            has("packed_color");
    gsm_ply_scene* s = new gsm_ply_scene();
    st = compressed ? load_compressed(data, size, h, (size_t)end, s) : load_standard(data, size, *vertex, (size_t)end, s);
    if (st != GSM_PLY_OK) {
        delete s;
        return st;
    }
    *out = s;
    return GSM_PLY_OK;
}

uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }  // Float16(x): nearest even

uint64_t expand_bits(uint64_t v) {  // expandBits (Scene.swift:48-56)
    uint64_t x = v & 0x1FFFFF;
    x = (x | (x << 32)) & 0x1F00000000FFFFull;
    x = (x | (x << 16)) & 0x1F0000FF0000FFull;
    x = (x | (x << 8)) & 0x100F00F00F00F00Full;
    x = (x | (x << 4)) & 0x10C30C30C30C30C3ull;
    x = (x | (x << 2)) & 0x1249249249249249ull;
    return x;
}

}  // namespace

extern "C" {

gsm_ply_status gsm_ply_load_memory(const void* bytes, size_t size, gsm_ply_scene** out) {
    if (!out) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "null output");
    *out = nullptr;
    if (!bytes && size) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "null input");
    return load_bytes((const uint8_t*)bytes, size, out);
}

gsm_ply_status gsm_ply_load(const char* path, gsm_ply_scene** out) {
    if (!out || !path) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return fail(GSM_PLY_ERR_IO, std::string("cannot open ") + path);
    const std::streamsize n = f.tellg();
    std::vector<uint8_t> buf((size_t)std::max<std::streamsize>(n, 0));
    f.seekg(0);
    if (n > 0 && !f.read((char*)buf.data(), n)) return fail(GSM_PLY_ERR_IO, std::string("cannot read ") + path);
    return load_bytes(buf.data(), buf.size(), out);
}

const char* gsm_ply_last_error(void) { return g_lastError.c_str(); }

const char* gsm_ply_status_string(gsm_ply_status s) {  // PLYLoaderError.errorDescription (:229-246)
    switch (s) {
        case GSM_PLY_OK: return "ok";
        case GSM_PLY_ERR_IO: return "Cannot read PLY file";
        case GSM_PLY_ERR_INVALID_HEADER: return "Invalid PLY header";
        case GSM_PLY_ERR_UNSUPPORTED_FORMAT: return "Unsupported PLY format";
        case GSM_PLY_ERR_MISSING_VERTEX_ELEMENT: return "Missing vertex element";
        case GSM_PLY_ERR_MISSING_REQUIRED_PROPERTIES: return "Missing required properties";
        case GSM_PLY_ERR_LIST_PROPERTIES_NOT_SUPPORTED: return "List properties are not supported";
        case GSM_PLY_ERR_INSUFFICIENT_DATA: return "Insufficient data in PLY file";
        case GSM_PLY_ERR_MISSING_CHUNK_ELEMENT: return "Missing chunk element in compressed PLY";
        case GSM_PLY_ERR_HEADER_FORMAT_MISSING: return "Header format missing";
        case GSM_PLY_ERR_HEADER_INVALID_CHARACTERS: return "Invalid characters in header";
        case GSM_PLY_ERR_HEADER_UNKNOWN_KEYWORD: return "Unknown keyword";
        case GSM_PLY_ERR_HEADER_UNEXPECTED_KEYWORD: return "Unexpected keyword";
        case GSM_PLY_ERR_HEADER_INVALID_LINE: return "Invalid line";
        case GSM_PLY_ERR_HEADER_INVALID_FORMAT_TYPE: return "Invalid format type";
        case GSM_PLY_ERR_HEADER_UNKNOWN_PROPERTY_TYPE: return "Unknown property type";
        case GSM_PLY_ERR_INVALID_ARGUMENT: return "Invalid argument";
    }
    return "unknown status";
}

void gsm_ply_free(gsm_ply_scene* s) { delete s; }
uint32_t gsm_ply_count(const gsm_ply_scene* s) { return s ? s->n : 0u; }
uint32_t gsm_ply_sh_components(const gsm_ply_scene* s) { return s ? s->shComponents : 0u; }
int gsm_ply_is_compressed(const gsm_ply_scene* s) { return s ? s->compressed : 0; }

gsm_ply_status gsm_ply_records(const gsm_ply_scene* s, float* positions, float* scales, float* rotations,
                               float* opacities, float* harmonics) {
    if (!s) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "null scene");
    if (positions) std::memcpy(positions, s->pos.data(), s->pos.size() * 4);
    if (scales) std::memcpy(scales, s->scale.data(), s->scale.size() * 4);
    if (rotations) std::memcpy(rotations, s->rot.data(), s->rot.size() * 4);
    if (opacities) std::memcpy(opacities, s->opacity.data(), s->opacity.size() * 4);
    if (harmonics) std::memcpy(harmonics, s->harmonics.data(), s->harmonics.size() * 4);
    return GSM_PLY_OK;
}

gsm_ply_status gsm_ply_bounds(const gsm_ply_scene* s, float center[3], float* radius) {
    // GaussianSceneBuilder.bounds(of:) (Scene.swift:172-196)
    if (!s || !center || !radius) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "null argument");
    if (s->n == 0) {
        center[0] = center[1] = center[2] = 0.0f;
        *radius = 1.0f;
        return GSM_PLY_OK;
    }
    float mn[3], mx[3];
    for (int c = 0; c < 3; ++c) mn[c] = mx[c] = s->pos[c];
    for (uint32_t i = 0; i < s->n; ++i)
        for (int c = 0; c < 3; ++c) {
            mn[c] = std::min(mn[c], s->pos[3 * i + c]);
            mx[c] = std::max(mx[c], s->pos[3 * i + c]);
        }
    for (int c = 0; c < 3; ++c) center[c] = (mn[c] + mx[c]) * 0.5f;
    auto len3 = [](float a, float b, float c) { return std::sqrt((a * a + b * b) + c * c); };
    float r = 0.0f;
    for (uint32_t i = 0; i < s->n; ++i) {
        const float* p = &s->pos[3 * i];
        const float* sc = &s->scale[3 * i];
        const float smax = std::max(sc[0], std::max(sc[1], sc[2]));
        r = std::max(r, len3(p[0] - center[0], p[1] - center[1], p[2] - center[2]) + smax);
    }
    r = std::max(r, len3(mx[0] - center[0], mx[1] - center[1], mx[2] - center[2]));
    *radius = std::max(r, 0.5f);
    return GSM_PLY_OK;
}

gsm_ply_status gsm_ply_sort_morton(gsm_ply_scene* s) {
    // GaussianSceneBuilder.sortByMortonCode (Scene.swift:74-138); stable for equal codes
    if (!s) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "null scene");
    const size_t n = s->n;
    if (n <= 1) return GSM_PLY_OK;
    float mn[3], mx[3];
    for (int c = 0; c < 3; ++c) mn[c] = mx[c] = s->pos[c];
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) {
            mn[c] = std::min(mn[c], s->pos[3 * i + c]);
            mx[c] = std::max(mx[c], s->pos[3 * i + c]);
        }
    float inv[3];
    for (int c = 0; c < 3; ++c) {
        const float ext = mx[c] - mn[c];
        inv[c] = ext > 1e-6f ? 1.0f / ext : 0.0f;
    }
    const float scale = (float)((1 << 21) - 1);
    std::vector<uint64_t> code(n);
    for (size_t i = 0; i < n; ++i) {
        uint64_t q[3];
        for (int c = 0; c < 3; ++c) {
            const float t = (s->pos[3 * i + c] - mn[c]) * inv[c];
            q[c] = (uint64_t)std::max(0.0f, std::min(scale, t * scale));
        }
        code[i] = expand_bits(q[0]) | (expand_bits(q[1]) << 1) | (expand_bits(q[2]) << 2);
    }
    std::vector<size_t> idx(n);
    for (size_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return code[a] < code[b]; });
    auto permute = [&](std::vector<float>& v, size_t w) {
        std::vector<float> o(v.size());
        for (size_t k = 0; k < n; ++k) std::memcpy(&o[k * w], &v[idx[k] * w], w * 4);
        v.swap(o);
    };
    permute(s->pos, 3);
    permute(s->scale, 3);
    permute(s->rot, 4);
    permute(s->opacity, 1);
    const size_t cpg = (size_t)s->shComponents * 3;
    if (cpg > 0 && s->harmonics.size() == n * cpg) permute(s->harmonics, cpg);
    return GSM_PLY_OK;
}

gsm_ply_status gsm_ply_packed_sizes(const gsm_ply_scene* s, int precision, size_t* gb, size_t* hb) {
    if (!s || !gb || !hb || (precision != 0 && precision != 1)) return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "bad argument");
    *gb = (size_t)s->n * (precision ? sizeof(gsm::PackedWorldGaussianHalf) : sizeof(gsm::PackedWorldGaussian));
    *hb = s->harmonics.size() * (precision ? 2u : 4u);
    return GSM_PLY_OK;
}

gsm_ply_status gsm_ply_pack(const gsm_ply_scene* s, int precision, void* gaussians, size_t gaussianBytes,
                            void* harmonics, size_t harmonicBytes) {
    size_t gb = 0, hb = 0;
    gsm_ply_status st = gsm_ply_packed_sizes(s, precision, &gb, &hb);
    if (st != GSM_PLY_OK) return st;
    if ((gb && (!gaussians || gaussianBytes < gb)) || (hb && (!harmonics || harmonicBytes < hb)))
        return fail(GSM_PLY_ERR_INVALID_ARGUMENT, "output buffer too small");
    // PackedWorldGaussian(Half).init(position:scale:rotation:opacity:) (KernelTypes.swift:12-53)
    for (uint32_t i = 0; i < s->n; ++i) {
        const float* p = &s->pos[3 * i];
        const float* sc = &s->scale[3 * i];
        const float* q = &s->rot[4 * i];
        if (precision) {
            gsm::PackedWorldGaussianHalf g;
            std::memset(&g, 0, sizeof(g));
            g.px = p[0];
            g.py = p[1];
            g.pz = p[2];
            g.opacity = f2h(s->opacity[i]);
            g.sx = f2h(sc[0]);
            g.sy = f2h(sc[1]);
            g.sz = f2h(sc[2]);
            g.rx = f2h(q[0]);
            g.ry = f2h(q[1]);
            g.rz = f2h(q[2]);
            g.rw = f2h(q[3]);
            std::memcpy((uint8_t*)gaussians + (size_t)i * sizeof(g), &g, sizeof(g));
        } else {
            gsm::PackedWorldGaussian g;
            std::memset(&g, 0, sizeof(g));
            g.px = p[0];
            g.py = p[1];
            g.pz = p[2];
            g.opacity = s->opacity[i];
            g.sx = sc[0];
            g.sy = sc[1];
            g.sz = sc[2];
            std::memcpy(g.rot, q, sizeof(g.rot));
            std::memcpy((uint8_t*)gaussians + (size_t)i * sizeof(g), &g, sizeof(g));
        }
    }
    // dataset.harmonics (.map(Float16.init) for half, PLYBenchmarkTests.swift:149)
    for (size_t k = 0; k < s->harmonics.size(); ++k) {
        if (precision) {
            const uint16_t h = f2h(s->harmonics[k]);
            std::memcpy((uint8_t*)harmonics + 2 * k, &h, 2);
        } else {
            std::memcpy((uint8_t*)harmonics + 4 * k, &s->harmonics[k], 4);
        }
    }
    return GSM_PLY_OK;
}

}  // extern "C"
