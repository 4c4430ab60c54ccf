// mesh_io.cpp — Wavefront OBJ and PLY triangle readers (see mesh_io.h).
#include "mesh_io.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <sstream>

namespace hippt {
namespace {

std::string lower_ext(const std::string &path) {
    const size_t dot = path.find_last_of('.');
    std::string e = dot == std::string::npos ? "" : path.substr(dot + 1);
    std::transform(e.begin(), e.end(), e.begin(), [](unsigned char c) { return char(std::tolower(c)); });
    return e;
}

bool fail(std::string &err, const std::string &path, long line, const std::string &msg) {
    err = path + (line > 0 ? ":" + std::to_string(line) : std::string()) + ": " + msg;
    return false;
}

// Fan triangulation of polygon `poly` (vertex indices) into out.verts.
void emit_fan(const std::vector<float> &pos, const std::vector<long> &poly, int group, MeshData &out) {
    for (size_t k = 1; k + 1 < poly.size(); ++k) {
        for (long v : {poly[0], poly[k], poly[k + 1]})
            out.verts.insert(out.verts.end(), pos.begin() + 3 * v, pos.begin() + 3 * v + 3);
        out.group.push_back(group);
    }
}

// ---- PLY -------------------------------------------------------------------------------------
enum class PlyType { I8, U8, I16, U16, I32, U32, F32, F64, Bad };

PlyType ply_type(const std::string &t) {
    if (t == "char" || t == "int8") return PlyType::I8;
    if (t == "uchar" || t == "uint8") return PlyType::U8;
    if (t == "short" || t == "int16") return PlyType::I16;
    if (t == "ushort" || t == "uint16") return PlyType::U16;
    if (t == "int" || t == "int32") return PlyType::I32;
    if (t == "uint" || t == "uint32") return PlyType::U32;
    if (t == "float" || t == "float32") return PlyType::F32;
    if (t == "double" || t == "float64") return PlyType::F64;
    return PlyType::Bad;
}

size_t ply_size(PlyType t) {
    switch (t) {
    case PlyType::I8:
    case PlyType::U8: return 1;
    case PlyType::I16:
    case PlyType::U16: return 2;
    case PlyType::I32:
    case PlyType::U32:
    case PlyType::F32: return 4;
    case PlyType::F64: return 8;
    default: return 0;
    }
}

struct PlyProp {
    std::string name;
    PlyType type = PlyType::Bad;
    bool list = false;
    PlyType countType = PlyType::Bad;
};

struct PlyElement {
    std::string name;
    long long count = 0;
    std::vector<PlyProp> props;
};

// Sequential value source over the body: ASCII tokens or binary (either byte order).
class PlyReader {
public:
    PlyReader(const std::vector<char> &body, int format) : b_(body), fmt_(format) {}
    // Reads one value of type t as double; false at end of data / malformed token.
    bool next(PlyType t, double &v) {
        if (fmt_ == 0) {
            while (pos_ < b_.size() && std::isspace(static_cast<unsigned char>(b_[pos_]))) ++pos_;
            if (pos_ >= b_.size()) return false;
            const size_t start = pos_;
            while (pos_ < b_.size() && !std::isspace(static_cast<unsigned char>(b_[pos_]))) ++pos_;
            const std::string tok(b_.data() + start, pos_ - start);
            char *end = nullptr;
            errno = 0;
            v = std::strtod(tok.c_str(), &end);
            return end && *end == '\0' && errno != ERANGE;
        }
        const size_t n = ply_size(t);
        if (n == 0 || pos_ + n > b_.size()) return false;
        unsigned char raw[8];
        std::memcpy(raw, b_.data() + pos_, n);
        pos_ += n;
        if (fmt_ == 2) std::reverse(raw, raw + n);  // big endian file on a little-endian host
        switch (t) {
        case PlyType::I8: v = double(int8_t(raw[0])); break;
        case PlyType::U8: v = double(raw[0]); break;
        case PlyType::I16: { int16_t x; std::memcpy(&x, raw, 2); v = x; break; }
        case PlyType::U16: { uint16_t x; std::memcpy(&x, raw, 2); v = x; break; }
        case PlyType::I32: { int32_t x; std::memcpy(&x, raw, 4); v = x; break; }
        case PlyType::U32: { uint32_t x; std::memcpy(&x, raw, 4); v = x; break; }
        case PlyType::F32: { float x; std::memcpy(&x, raw, 4); v = x; break; }
        case PlyType::F64: { double x; std::memcpy(&x, raw, 8); v = x; break; }
        default: return false;
        }
        return true;
    }

private:
    const std::vector<char> &b_;
    int fmt_;  // 0 ascii, 1 little endian, 2 big endian
    size_t pos_ = 0;
};

}  // namespace

bool read_obj(const std::string &path, MeshData &out, std::string &err) {
    std::ifstream f(path);
    if (!f) return fail(err, path, 0, "cannot open");
    out = MeshData();
    std::vector<float> pos;
    std::map<std::string, int> groupIndex;
    std::string current;  // material of the following faces ("" until the first usemtl)
    std::vector<long> poly;
    std::string line;
    long lineNo = 0;
    while (std::getline(f, line)) {
        ++lineNo;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream in(line);
        std::string key;
        if (!(in >> key) || key[0] == '#') continue;
        if (key == "v") {
            std::string tok[3];
            if (!(in >> tok[0] >> tok[1] >> tok[2])) return fail(err, path, lineNo, "vertex needs x y z");
            for (const std::string &t : tok) {
                char *end = nullptr;
                const float x = std::strtof(t.c_str(), &end);  // correctly rounded to float
                if (!end || *end != '\0' || !std::isfinite(x)) return fail(err, path, lineNo, "bad coordinate '" + t + "'");
                pos.push_back(x);
            }
        } else if (key == "f") {
            poly.clear();
            const long nv = long(pos.size() / 3);
            std::string tok;
            while (in >> tok) {
                char *end = nullptr;
                const long i = std::strtol(tok.c_str(), &end, 10);  // v, v/vt, v//vn, v/vt/vn
                if (end == tok.c_str() || (*end != '\0' && *end != '/') || i == 0)
                    return fail(err, path, lineNo, "bad face index '" + tok + "'");
                const long v = i > 0 ? i - 1 : nv + i;  // negative: relative to the end
                if (v < 0 || v >= nv) return fail(err, path, lineNo, "face index out of range '" + tok + "'");
                poly.push_back(v);
            }
            if (poly.size() < 3) return fail(err, path, lineNo, "face needs at least 3 vertices");
            auto it = groupIndex.find(current);
            if (it == groupIndex.end()) {
                it = groupIndex.emplace(current, int(out.groups.size())).first;
                out.groups.push_back(current);
            }
            emit_fan(pos, poly, it->second, out);
        } else if (key == "usemtl") {
            std::string name;
            std::getline(in >> std::ws, name);
            current = name;
        }
        // vt, vn, vp, o, g, s, mtllib, l, p: not needed for closest-hit geometry
    }
    if (out.group.empty()) return fail(err, path, 0, "no faces");
    return true;
}

bool read_ply(const std::string &path, MeshData &out, std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(err, path, 0, "cannot open");
    out = MeshData();
    std::string line;
    long lineNo = 0;
    int format = -1;
    std::vector<PlyElement> elems;
    bool ended = false;
    while (std::getline(f, line)) {
        ++lineNo;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream in(line);
        std::string key;
        in >> key;
        if (lineNo == 1) {
            if (key != "ply") return fail(err, path, 1, "not a PLY file");
            continue;
        }
        if (key == "format") {
            std::string fmt;
            in >> fmt;
            format = fmt == "ascii" ? 0 : fmt == "binary_little_endian" ? 1 : fmt == "binary_big_endian" ? 2 : -1;
            if (format < 0) return fail(err, path, lineNo, "unknown format '" + fmt + "'");
        } else if (key == "element") {
            PlyElement e;
            if (!(in >> e.name >> e.count) || e.count < 0) return fail(err, path, lineNo, "bad element line");
            elems.push_back(e);
        } else if (key == "property") {
            if (elems.empty()) return fail(err, path, lineNo, "property before element");
            PlyProp p;
            std::string t;
            in >> t;
            if (t == "list") {
                std::string ct, it;
                in >> ct >> it >> p.name;
                p.list = true;
                p.countType = ply_type(ct);
                p.type = ply_type(it);
                if (p.countType == PlyType::Bad || p.type == PlyType::Bad)
                    return fail(err, path, lineNo, "bad list property types");
            } else {
                p.type = ply_type(t);
                in >> p.name;
                if (p.type == PlyType::Bad) return fail(err, path, lineNo, "bad property type '" + t + "'");
            }
            elems.back().props.push_back(p);
        } else if (key == "end_header") {
            ended = true;
            break;
        }
        // comment, obj_info: ignored
    }
    if (!ended || format < 0) return fail(err, path, lineNo, "incomplete header");
    std::vector<char> body((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    PlyReader rd(body, format);
    std::vector<float> pos;
    std::vector<long> poly;
    for (const PlyElement &e : elems) {
        int ix = -1, iy = -1, iz = -1, iface = -1;
        for (int k = 0; k < int(e.props.size()); ++k) {
            const PlyProp &p = e.props[size_t(k)];
            if (!p.list && p.name == "x") ix = k;
            if (!p.list && p.name == "y") iy = k;
            if (!p.list && p.name == "z") iz = k;
            if (p.list && (p.name == "vertex_indices" || p.name == "vertex_index")) iface = k;
        }
        const bool isVertex = e.name == "vertex", isFace = e.name == "face";
        if (isVertex && (ix < 0 || iy < 0 || iz < 0)) return fail(err, path, 0, "vertex element without x, y, z");
        if (isFace && iface < 0) return fail(err, path, 0, "face element without vertex_indices");
        const long nv = long(pos.size() / 3);
        for (long long r = 0; r < e.count; ++r) {
            float xyz[3] = {0, 0, 0};
            poly.clear();
            for (int k = 0; k < int(e.props.size()); ++k) {
                const PlyProp &p = e.props[size_t(k)];
                double v;
                if (p.list) {
                    if (!rd.next(p.countType, v) || v < 0) return fail(err, path, 0, "truncated or bad list count");
                    const long n = long(v);
                    for (long j = 0; j < n; ++j) {
                        if (!rd.next(p.type, v)) return fail(err, path, 0, "truncated list");
                        if (isFace && k == iface) {
                            if (v < 0 || v >= double(nv) || v != std::floor(v))
                                return fail(err, path, 0, "face index out of range");
                            poly.push_back(long(v));
                        }
                    }
                } else {
                    if (!rd.next(p.type, v)) return fail(err, path, 0, "truncated " + e.name + " data");
                    if (isVertex && (k == ix || k == iy || k == iz)) {
                        const float x = float(v);
                        if (!std::isfinite(x)) return fail(err, path, 0, "non-finite vertex coordinate");
                        xyz[k == ix ? 0 : k == iy ? 1 : 2] = x;
                    }
                }
            }
            if (isVertex) pos.insert(pos.end(), xyz, xyz + 3);
            if (isFace) {
                if (poly.size() < 3) return fail(err, path, 0, "face needs at least 3 vertices");
                emit_fan(pos, poly, 0, out);
            }
        }
    }
    if (out.group.empty()) return fail(err, path, 0, "no faces");
    out.groups.assign(1, "");
    return true;
}

bool read_mesh(const std::string &path, MeshData &out, std::string &err) {
    const std::string e = lower_ext(path);
    if (e == "obj") return read_obj(path, out, err);
    if (e == "ply") return read_ply(path, out, err);
    return fail(err, path, 0, "unknown mesh format (expected .obj or .ply)");
}

}  // namespace hippt
