// pbr_host.cpp — the C++ host API of include/pbr/pbr.h: the reference's scene classes, flattened
// into a pbr_scene_desc and rendered through the C-ABI (include/pbr_hip.h).
#include "../../include/pbr/pbr.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <unordered_map>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "../../include/pbr_hip.h"
#include <type_traits>
#include "../csrc/pbr_xform.h"

// ============================================================================ FrameBuffer
void FrameBuffer::InitBuffer(int w, int h, int ch) {
    width = w;
    height = h;
    channals = ch;
    ubuffer.clear();
    fbuffer.clear();
    if (ch > 4 || w <= 0 || h <= 0) return;
    ubuffer.assign((size_t)w * h * ch, 0);
    fbuffer.assign((size_t)w * h * ch, 0.f);
}
void FrameBuffer::FreeBuffer() {
    ubuffer.clear();
    fbuffer.clear();
    width = height = channals = 0;
}
bool FrameBuffer::bufferResize(int w, int h) {
    if (width == 0 || height == 0 || channals == 0) return false;
    InitBuffer(w, h, channals);
    return true;
}
bool FrameBuffer::set_uc(int w, int h, int shifting, const unsigned char& dat) {
    if (ubuffer.empty() || w >= width || h >= height || w < 0 || h < 0) return false;
    ubuffer[((size_t)w + (size_t)h * width) * channals + shifting] = dat;
    return true;
}
bool FrameBuffer::set_fc(int w, int h, int shifting, const float& dat) {
    if (fbuffer.empty() || w >= width || h >= height || w < 0 || h < 0) return false;
    fbuffer[((size_t)w + (size_t)h * width) * channals + shifting] = dat;
    return true;
}

bool FrameBuffer::update_f_u_c(int w, int h, int shifting, int renderCount, const float& dat) {
    if (fbuffer.empty() || w >= width || h >= height || w < 0 || h < 0) return false;
    const size_t off = ((size_t)w + (size_t)h * width) * channals + shifting;
    float weight = (1.0f / (float)renderCount);
    fbuffer[off] = weight * dat + (1.0f - weight) * fbuffer[off];
    ubuffer[off] = (unsigned char)(fbuffer[off] * 255);
    return true;
}

namespace {
int g_flip_on_write = 0;
uint32_t png_crc(const unsigned char* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
            table[i] = c;
        }
        init = true;
    }
    uint32_t c = 0xffffffffu;
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xffu] ^ (c >> 8);
    return c ^ 0xffffffffu;
}
void put_be32(std::vector<unsigned char>& o, uint32_t v) {
    o.push_back((unsigned char)(v >> 24)); o.push_back((unsigned char)(v >> 16));
    o.push_back((unsigned char)(v >> 8)); o.push_back((unsigned char)v);
}
void put_chunk(std::vector<unsigned char>& o, const char* type, const std::vector<unsigned char>& data) {
    put_be32(o, (uint32_t)data.size());
    const size_t start = o.size();
    o.insert(o.end(), type, type + 4);
    o.insert(o.end(), data.begin(), data.end());
    put_be32(o, png_crc(&o[start], o.size() - start));
}
}  // namespace

void stbi_flip_vertically_on_write(int flag) { g_flip_on_write = flag; }

int stbi_write_png(char const* filename, int w, int h, int comp, const void* data, int stride_in_bytes) {
    if (!filename || !data || w <= 0 || h <= 0 || comp < 1 || comp > 4) return 0;
    static const unsigned char kColorType[5] = {0, 0, 4, 2, 6};   // grey, grey+alpha, RGB, RGBA
    const size_t row = (size_t)w * comp;
    const size_t stride = stride_in_bytes ? (size_t)stride_in_bytes : row;
    const unsigned char* px = (const unsigned char*)data;
    // scanlines, each behind filter byte 0 (None)
    std::vector<unsigned char> raw;
    raw.reserve((size_t)h * (row + 1));
    for (int y = 0; y < h; ++y) {
        const unsigned char* src = px + (size_t)(g_flip_on_write ? h - 1 - y : y) * stride;
        raw.push_back(0);
        raw.insert(raw.end(), src, src + row);
    }
    // zlib stream: header, stored deflate blocks of at most 65535 bytes, Adler-32
    std::vector<unsigned char> z = {0x78, 0x01};
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        z.push_back(pos + n == raw.size() ? 1 : 0);
        z.push_back((unsigned char)(n & 0xff)); z.push_back((unsigned char)(n >> 8));
        z.push_back((unsigned char)(~n & 0xff)); z.push_back((unsigned char)((~n >> 8) & 0xff));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (unsigned char c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
    put_be32(z, b << 16 | a);
    std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<unsigned char> ihdr;
    put_be32(ihdr, (uint32_t)w);
    put_be32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, kColorType[comp], 0, 0, 0});   // depth, color type, deflate, filter 0, no interlace
    put_chunk(out, "IHDR", ihdr);
    put_chunk(out, "IDAT", z);
    put_chunk(out, "IEND", {});
    FILE* f = std::fopen(filename, "wb");
    if (!f) return 0;
    const size_t wr = std::fwrite(out.data(), 1, out.size(), f);
    return (std::fclose(f) == 0 && wr == out.size()) ? 1 : 0;
}

namespace PBR {

namespace {

pbr::xform::Mat to_mat(const Matrix4x4& m) {
    pbr::xform::Mat r;
    std::memcpy(r.a, m.m, 64);
    return r;
}
Matrix4x4 from_mat(const pbr::xform::Mat& m) { return Matrix4x4(m.a); }
Transform from_xf(const pbr::xform::Xf& x) { return Transform(from_mat(x.m), from_mat(x.mi)); }
pbr::f3 f3of(const Vector3f& v) { return pbr::mk(v.x, v.y, v.z); }

void fill_transform(const Transform& t, pbr_transform* out) {
    std::memcpy(out->m, t.GetMatrix().m, 64);
    std::memcpy(out->m_inv, t.GetInverseMatrix().m, 64);
}

std::atomic<uint64_t> g_sceneIds{1};

}  // namespace

// ============================================================================ Transform
Matrix4x4::Matrix4x4() {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) m[i][j] = i == j ? 1.f : 0.f;
}
Matrix4x4::Matrix4x4(const float mat[4][4]) { std::memcpy(m, mat, 64); }
Matrix4x4::Matrix4x4(float t00, float t01, float t02, float t03, float t10, float t11, float t12, float t13, float t20,
                     float t21, float t22, float t23, float t30, float t31, float t32, float t33) {
    const float v[16] = {t00, t01, t02, t03, t10, t11, t12, t13, t20, t21, t22, t23, t30, t31, t32, t33};
    std::memcpy(m, v, 64);
}
Matrix4x4 Inverse(const Matrix4x4& m) { return from_mat(pbr::xform::invert(to_mat(m))); }
Matrix4x4 Mul(const Matrix4x4& a, const Matrix4x4& b) { return from_mat(pbr::xform::mul(to_mat(a), to_mat(b))); }
Transform::Transform(const float mat[4][4]) : m(mat), mInv(Inverse(m)) {}
Transform::Transform(const Matrix4x4& m) : m(m), mInv(Inverse(m)) {}
Transform Transform::operator*(const Transform& t2) const { return Transform(Mul(m, t2.m), Mul(t2.mInv, mInv)); }

Transform Translate(const Vector3f& d) { return from_xf(pbr::xform::translate(f3of(d))); }
Transform Scale(float x, float y, float z) { return from_xf(pbr::xform::scale(x, y, z)); }
namespace {
Transform rotate_axis(float theta, int axis) {   // Transform.cpp RotateX/Y/Z: m and its transpose
    float rad = (pbr::kPi / 180) * theta;
    float s = pbr::t_sin(rad), c = pbr::t_cos(rad);
    Matrix4x4 m;
    int a = (axis + 1) % 3, b = (axis + 2) % 3;
    m.m[a][a] = c;
    m.m[b][b] = c;
    // RotateX: m[1][2] = -s, m[2][1] = s; RotateY: m[0][2] = s, m[2][0] = -s; RotateZ: m[0][1] = -s, m[1][0] = s
    if (axis == 1) { m.m[0][2] = s; m.m[2][0] = -s; }
    else { m.m[a][b] = -s; m.m[b][a] = s; }
    Matrix4x4 t;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) t.m[i][j] = m.m[j][i];
    return Transform(m, t);
}
}  // namespace
Transform RotateX(float theta) { return rotate_axis(theta, 0); }
Transform RotateY(float theta) { return rotate_axis(theta, 1); }
Transform RotateZ(float theta) { return rotate_axis(theta, 2); }
Transform LookAt(const Point3f& pos, const Point3f& look, const Vector3f& up) {
    return from_xf(pbr::xform::look_at(f3of(pos), f3of(look), f3of(up)));
}

// ============================================================================ shapes
TriangleMesh::TriangleMesh(const Transform& ObjectToWorld, int nTriangles, const int* vi, int nVertices, const Point3f* P,
                           const Vector3f* /*S*/, const Normal3f* N, const Point2f* UV, const int* /*faceIndices*/)
    : nTriangles(nTriangles), nVertices(nVertices), objectToWorld(ObjectToWorld), vertexIndices(vi, vi + 3 * nTriangles) {
    p.resize((size_t)3 * nVertices);
    for (int i = 0; i < nVertices; ++i) { p[3 * i] = P[i].x; p[3 * i + 1] = P[i].y; p[3 * i + 2] = P[i].z; }
    if (N) {
        n.resize((size_t)3 * nVertices);
        for (int i = 0; i < nVertices; ++i) { n[3 * i] = N[i].x; n[3 * i + 1] = N[i].y; n[3 * i + 2] = N[i].z; }
    }
    if (UV) {
        uv.resize((size_t)2 * nVertices);
        for (int i = 0; i < nVertices; ++i) { uv[2 * i] = UV[i].x; uv[2 * i + 1] = UV[i].y; }
    }
}

std::vector<std::shared_ptr<Shape>> CreateTriangleMesh(const Transform* o2w, const Transform* w2o, bool reverseOrientation,
                                                       int nTriangles, const int* vertexIndices, int nVertices,
                                                       const Point3f* p, const Vector3f* s, const Normal3f* n,
                                                       const Point2f* uv, const int* faceIndices) {
    auto mesh = std::make_shared<TriangleMesh>(*o2w, nTriangles, vertexIndices, nVertices, p, s, n, uv, faceIndices);
    std::vector<std::shared_ptr<Shape>> tris;
    tris.reserve(nTriangles);
    for (int i = 0; i < nTriangles; ++i) tris.push_back(std::make_shared<Triangle>(o2w, w2o, reverseOrientation, mesh, i));
    return tris;
}

plyInfo::plyInfo(const std::string& filePath) {   // Shape/plyRead.h:22-47
    std::ifstream f(filePath);
    if (!f) throw std::runtime_error("plyInfo: cannot open " + filePath);
    std::string ed;
    for (int i = 0; i < 2; i++) {
        f >> ed;
        if (ed == "vertex") f >> nVertices;
        else if (ed == "face") f >> nTriangles;
    }
    vertexArray.resize(nVertices);
    vertexIndices.resize((size_t)3 * nTriangles);
    for (int i = 0; i < nVertices; i++) {
        f >> vertexArray[i].x >> vertexArray[i].y >> vertexArray[i].z;
        vertexArray[i].x *= 20; vertexArray[i].y *= 20; vertexArray[i].z *= 20;
    }
    for (int i = 0; i < nTriangles; i++) f >> ed >> vertexIndices[i * 3] >> vertexIndices[i * 3 + 1] >> vertexIndices[i * 3 + 2];
    if (!f) throw std::runtime_error("plyInfo: truncated " + filePath);
}

namespace {
struct PlyProp { std::string name, type, countType; bool list = false; };
struct PlyElem { std::string name; long count = 0; std::vector<PlyProp> props; };
size_t ply_size(const std::string& t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    throw std::runtime_error("LoadPLY: unknown property type " + t);
}
double ply_read_bin(const unsigned char* b, const std::string& t) {
    if (t == "char" || t == "int8") return (double)*(const int8_t*)b;
    if (t == "uchar" || t == "uint8") return (double)*b;
    int16_t s; uint16_t us; int32_t i; uint32_t u; float fl; double d;
    if (t == "short" || t == "int16") { std::memcpy(&s, b, 2); return s; }
    if (t == "ushort" || t == "uint16") { std::memcpy(&us, b, 2); return us; }
    if (t == "int" || t == "int32") { std::memcpy(&i, b, 4); return i; }
    if (t == "uint" || t == "uint32") { std::memcpy(&u, b, 4); return u; }
    if (t == "float" || t == "float32") { std::memcpy(&fl, b, 4); return fl; }
    std::memcpy(&d, b, 8);
    return d;
}
}  // namespace

PlyMesh LoadPLY(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("LoadPLY: cannot open " + path);
    std::string line, format;
    std::vector<PlyElem> elems;
    std::getline(f, line);
    if (line.rfind("ply", 0) != 0) throw std::runtime_error("LoadPLY: not a PLY file");
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ls(line);
        std::string kw;
        ls >> kw;
        if (kw == "format") ls >> format;
        else if (kw == "element") { PlyElem e; ls >> e.name >> e.count; elems.push_back(e); }
        else if (kw == "property") {
            PlyProp p;
            std::string t;
            ls >> t;
            if (t == "list") { p.list = true; ls >> p.countType >> p.type >> p.name; }
            else { p.type = t; ls >> p.name; }
            if (elems.empty()) throw std::runtime_error("LoadPLY: property before element");
            elems.back().props.push_back(p);
        } else if (kw == "end_header") break;
    }
    if (format != "ascii" && format != "binary_little_endian") throw std::runtime_error("LoadPLY: unsupported format " + format);
    const bool ascii = format == "ascii";
    PlyMesh out;
    for (const PlyElem& e : elems) {
        int ix = -1, iy = -1, iz = -1, iface = -1;
        for (size_t k = 0; k < e.props.size(); ++k) {
            if (e.props[k].name == "x") ix = (int)k;
            if (e.props[k].name == "y") iy = (int)k;
            if (e.props[k].name == "z") iz = (int)k;
            if (e.props[k].list && (e.props[k].name == "vertex_indices" || e.props[k].name == "vertex_index")) iface = (int)k;
        }
        for (long r = 0; r < e.count; ++r) {
            std::vector<double> scalars(e.props.size(), 0.0);
            std::vector<long> face;
            for (size_t k = 0; k < e.props.size(); ++k) {
                const PlyProp& p = e.props[k];
                if (p.list) {
                    long cnt;
                    if (ascii) f >> cnt;
                    else { unsigned char b[8]; f.read((char*)b, ply_size(p.countType)); cnt = (long)ply_read_bin(b, p.countType); }
                    for (long c = 0; c < cnt; ++c) {
                        double v;
                        if (ascii) f >> v;
                        else { unsigned char b[8]; f.read((char*)b, ply_size(p.type)); v = ply_read_bin(b, p.type); }
                        if ((int)k == iface) face.push_back((long)v);
                    }
                } else {
                    if (ascii) f >> scalars[k];
                    else { unsigned char b[8]; f.read((char*)b, ply_size(p.type)); scalars[k] = ply_read_bin(b, p.type); }
                }
            }
            if (!f) throw std::runtime_error("LoadPLY: truncated " + path);
            if (e.name == "vertex" && ix >= 0 && iy >= 0 && iz >= 0)
                out.vertices.emplace_back((float)scalars[ix], (float)scalars[iy], (float)scalars[iz]);
            if (e.name == "face" && iface >= 0)
                for (size_t k = 2; k < face.size(); ++k) {   // fan-triangulate quads / polygons
                    out.indices.push_back((int)face[0]);
                    out.indices.push_back((int)face[k - 1]);
                    out.indices.push_back((int)face[k]);
                }
        }
    }
    return out;
}

// ============================================================================ lights
namespace {
// Radiance RGBE → float exactly as stbi_loadf (stbi__hdr_load / stbi__hdr_convert), rows flipped
// as stbi_set_flip_vertically_on_load(true) does (SkyBoxLight.cpp:19-24).
// stb's global stbi_set_flip_vertically_on_load flag: SkyBoxLight::loadImage sets it (and it stays set)
bool g_stbiFlip = false;
bool load_hdr(const char* file, int* w, int* h, int* comp, std::vector<float>* data, bool flip) {
    std::ifstream f(file, std::ios::binary);
    if (!f) return false;
    std::string line;
    std::getline(f, line);
    if (line != "#?RADIANCE" && line != "#?RGBE") return false;
    bool fmt = false;
    while (std::getline(f, line)) {
        if (line.empty()) break;
        if (line == "FORMAT=32-bit_rle_rgbe") fmt = true;
    }
    if (!fmt) return false;
    std::getline(f, line);
    int H = 0, W = 0;
    if (std::sscanf(line.c_str(), "-Y %d +X %d", &H, &W) != 2 || W <= 0 || H <= 0) return false;
    std::vector<unsigned char> rgbe((size_t)W * H * 4);
    auto rd = [&](unsigned char* p, size_t n) { f.read((char*)p, (std::streamsize)n); return (bool)f; };
    bool flat = W < 8 || W >= 32768;
    for (int y = 0; y < H && !flat; ++y) {
        unsigned char hdr[4];
        if (!rd(hdr, 4)) return false;
        if (hdr[0] != 2 || hdr[1] != 2 || (hdr[2] & 0x80)) {   // not RLE: these 4 bytes are the first pixel
            if (y != 0) return false;
            std::memcpy(&rgbe[0], hdr, 4);
            if (!rd(&rgbe[4], rgbe.size() - 4)) return false;
            flat = true;
            break;
        }
        if (((int)hdr[2] << 8 | hdr[3]) != W) return false;
        std::vector<unsigned char> sc((size_t)W * 4);
        for (int c = 0; c < 4; ++c) {
            int i = 0;
            while (i < W) {
                unsigned char cnt;
                if (!rd(&cnt, 1)) return false;
                if (cnt > 128) {
                    unsigned char v;
                    if (!rd(&v, 1)) return false;
                    cnt -= 128;
                    if (i + cnt > W) return false;
                    for (int k = 0; k < cnt; ++k) sc[(size_t)(i++) * 4 + c] = v;
                } else {
                    if (cnt == 0 || i + cnt > W) return false;
                    for (int k = 0; k < cnt; ++k) { unsigned char v; if (!rd(&v, 1)) return false; sc[(size_t)(i++) * 4 + c] = v; }
                }
            }
        }
        std::memcpy(&rgbe[(size_t)y * W * 4], sc.data(), sc.size());
        if (y == H - 1) break;
    }
    if (flat && W >= 8 && W < 32768 && rgbe.empty()) return false;
    if (flat && (W < 8 || W >= 32768) && !rd(rgbe.data(), rgbe.size())) return false;
    data->assign((size_t)W * H * 3, 0.f);
    for (int y = 0; y < H; ++y) {
        int dy = flip ? H - 1 - y : y;   // vertical flip
        for (int x = 0; x < W; ++x) {
            const unsigned char* in = &rgbe[((size_t)y * W + x) * 4];
            float* o = &(*data)[((size_t)dy * W + x) * 3];
            if (in[3] != 0) {
                float f1 = (float)std::ldexp(1.0f, in[3] - (int)(128 + 8));
                o[0] = in[0] * f1; o[1] = in[1] * f1; o[2] = in[2] * f1;
            }
        }
    }
    *w = W; *h = H; *comp = 3;
    return true;
}
}  // namespace

// ============================================================================ ImageTexture
template <typename Tmemory, typename Treturn>
ImageTexture<Tmemory, Treturn>::ImageTexture(std::unique_ptr<TextureMapping2D> m, const std::string& filename, bool doTrilinear,
                                             float maxAniso, ImageWrap wrapMode, float scale, bool gamma)
    : mapping(std::move(m)) {
    img.mapping = dynamic_cast<const UVMapping2D*>(mapping.get());
    img.doTrilinear = doTrilinear; img.maxAniso = maxAniso; img.wrapMode = wrapMode; img.scale = scale; img.gamma = gamma;
    img.isFloat = std::is_same<Tmemory, float>::value;
    g_stbiFlip = true;   // loadImage: stbi_set_flip_vertically_on_load(true), left set
    if (filename.empty() || !load_hdr(filename.c_str(), &img.width, &img.height, &img.components, &img.data, true)) {
        img.width = img.height = img.components = 0;
        img.data.clear();
    }
}
template <typename Tmemory, typename Treturn>
ImageTexture<Tmemory, Treturn>::ImageTexture(std::unique_ptr<TextureMapping2D> m, int width, int height, int components,
                                             std::vector<float> data, bool doTrilinear, float maxAniso, ImageWrap wrapMode,
                                             float scale, bool gamma)
    : mapping(std::move(m)) {
    if (!data.empty() && (width <= 0 || height <= 0 || components < 3 || data.size() != (size_t)width * height * components))
        throw std::invalid_argument("ImageTexture: bad image");
    img.mapping = dynamic_cast<const UVMapping2D*>(mapping.get());
    img.width = width; img.height = height; img.components = components; img.data = std::move(data);
    img.doTrilinear = doTrilinear; img.maxAniso = maxAniso; img.wrapMode = wrapMode; img.scale = scale; img.gamma = gamma;
    img.isFloat = std::is_same<Tmemory, float>::value;
}
template class ImageTexture<RGBSpectrum, Spectrum>;
template class ImageTexture<float, float>;

SkyBoxLight::SkyBoxLight(const Transform& LightToWorld, const Point3f& worldCenter, float worldRadius, const char* file, int nSamples)
    : Light(LightToWorld, MediumInterface(), nSamples), worldCenter(worldCenter), worldRadius(worldRadius) {
    loadImage(file);   // as the reference: a missing file leaves a black sky
}
SkyBoxLight::SkyBoxLight(const Transform& LightToWorld, const Point3f& worldCenter, float worldRadius, int width, int height,
                         int components, std::vector<float> d, int nSamples)
    : Light(LightToWorld, MediumInterface(), nSamples), worldCenter(worldCenter), worldRadius(worldRadius),
      imageWidth(width), imageHeight(height), nrComponents(components), data(std::move(d)) {
    if ((size_t)width * height * components != data.size()) throw std::invalid_argument("SkyBoxLight: data size mismatch");
}
bool SkyBoxLight::loadImage(const char* imageFile) {
    imageWidth = imageHeight = nrComponents = 0;
    data.clear();
    g_stbiFlip = true;   // stbi_set_flip_vertically_on_load(true)
    return imageFile && load_hdr(imageFile, &imageWidth, &imageHeight, &nrComponents, &data, true);
}
InfiniteAreaLight::InfiniteAreaLight(const Transform& LightToWorld, const Spectrum& power, int nSamples, const std::string& texmap)
    : Light(LightToWorld, MediumInterface(), nSamples), L(power) {
    if (!texmap.empty() && !load_hdr(texmap.c_str(), &imageWidth, &imageHeight, &nrComponents, &data, g_stbiFlip)) {
        imageWidth = imageHeight = nrComponents = 0;
        data.clear();
    }
}
InfiniteAreaLight::InfiniteAreaLight(const Transform& LightToWorld, const Spectrum& power, int nSamples, int width,
                                     int height, int components, std::vector<float> d)
    : Light(LightToWorld, MediumInterface(), nSamples), L(power), imageWidth(width), imageHeight(height),
      nrComponents(components), data(std::move(d)) {
    if ((size_t)width * height * components != data.size()) throw std::invalid_argument("InfiniteAreaLight: data size mismatch");
}

// ============================================================================ aggregate, scene, camera, sampler
BVHAccel::BVHAccel(std::vector<std::shared_ptr<Primitive>> p, int maxPrimsInNode, SplitMethod splitMethod)
    : maxPrimsInNode(std::min(255, maxPrimsInNode)), splitMethod(splitMethod), primitives(std::move(p)) {
    // BVHAccel.cpp:131-160: the reference's switch has no HLBVH branch, so HLBVH builds with SAH;
    // Middle and EqualCounts are flattened as such (pbr_scene_desc.split_method) and built on the host
}

Bounds3f::Bounds3f() {
    const float M = 3.40282347e+38f;
    pMin = Point3f(M, M, M);
    pMax = Point3f(-M, -M, -M);
}

const Medium* SurfaceInteraction::GetMedium(const Vector3f& w) const {
    const float d = w.x * n.x + w.y * n.y + w.z * n.z;
    return d > 0 ? mediumInterface.outside : mediumInterface.inside;
}

// ---- device-side queries of a Scene (pbr_hip_query / pbr_hip_bounds on the scene's own context)
struct SceneDevice {
    pbr_hip_ctx* ctx = nullptr;
    std::shared_ptr<FlatScene> flat;
    std::vector<const Primitive*> prims;   // the BVHAccel's primitive vector
    Bounds3f worldBound;
    ~SceneDevice() {
        if (ctx) pbr_hip_destroy(ctx);
    }
};

Scene::Scene(std::shared_ptr<Primitive> aggregate, const std::vector<std::shared_ptr<Light>>& lights)
    : lights(lights), aggregate(std::move(aggregate)), id(g_sceneIds++) {
    for (const auto& l : lights)
        if (l->IsInfinite()) infiniteLights.push_back(l);
    // the primitives answer their own queries through this scene's device context
    if (auto* bvh = dynamic_cast<const BVHAccel*>(this->aggregate.get())) {
        bvh->owner = this;
        int k = 0;
        for (const auto& p : bvh->Primitives()) {
            if (auto* gp = dynamic_cast<const GeometricPrimitive*>(p.get())) { gp->owner = this; gp->ownerIndex = k; }
            ++k;
        }
    }
}

Scene::~Scene() {
    if (auto* bvh = dynamic_cast<const BVHAccel*>(aggregate.get())) {
        if (bvh->owner == this) bvh->owner = nullptr;
        for (const auto& p : bvh->Primitives())
            if (auto* gp = dynamic_cast<const GeometricPrimitive*>(p.get()))
                if (gp->owner == this) { gp->owner = nullptr; gp->ownerIndex = -1; }
    }
}

PerspectiveCamera::PerspectiveCamera(int RasterWidth, int RasterHeight, const Transform& CameraToWorld, const Bounds2f& screenWindow,
                                     float lensRadius, float focalDistance, float fov, const Medium* medium)
    : RasterWidth(RasterWidth), RasterHeight(RasterHeight), CameraToWorld(CameraToWorld), screenWindow(screenWindow),
      lensRadius(lensRadius), focalDistance(focalDistance), fov(fov), medium(medium) {}

PerspectiveCamera* CreatePerspectiveCamera(int RasterWidth, int RasterHeight, const Transform& cam2world, Medium* media) {
    // Camera/Perspective.cpp:84-104
    float frame = (float)RasterWidth / (float)RasterHeight;
    Bounds2f screen;
    if (frame > 1.f) { screen.pMin.x = -frame; screen.pMax.x = frame; screen.pMin.y = -1.f; screen.pMax.y = 1.f; }
    else { screen.pMin.x = -1.f; screen.pMax.x = 1.f; screen.pMin.y = -1.f / frame; screen.pMax.y = 1.f / frame; }
    return new PerspectiveCamera(RasterWidth, RasterHeight, cam2world, screen, 0.0f, 0.0f, 90.0f, media);
}

HaltonSampler::HaltonSampler(int nsamp, const Bounds2i& sampleBounds, bool sampleAtCenter)
    : GlobalSampler(nsamp), sampleBounds(sampleBounds) {
    if (sampleAtCenter) throw std::invalid_argument("HaltonSampler: sampleAtCenter is not on the GPU path");
}
HaltonSampler* CreateHaltonSampler(const Bounds2i& sampleBounds) { return new HaltonSampler(16, sampleBounds, false); }
std::unique_ptr<Sampler> HaltonSampler::Clone(int) { return std::unique_ptr<Sampler>(new HaltonSampler(*this)); }
int HaltonSampler::DeviceSampler() const { return PBR_SAMPLER_HALTON; }
Point2i HaltonSampler::SampleRaster() const {
    return Point2i(sampleBounds.pMax.x - sampleBounds.pMin.x, sampleBounds.pMax.y - sampleBounds.pMin.y);
}
namespace {
void check(pbr_hip_ctx* ctx, int rc, const char* what);
pbr_hip_ctx* helper_ctx();
int64_t round_up_pow2(int64_t v) {
    int64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}
}  // namespace
SobolSampler::SobolSampler(int64_t samplesPerPixel, const Bounds2i& sampleBounds)
    : GlobalSampler(round_up_pow2(samplesPerPixel)), sampleBounds(sampleBounds) {
    if (samplesPerPixel <= 0) throw std::invalid_argument("SobolSampler: samplesPerPixel must be positive");
}
std::unique_ptr<Sampler> SobolSampler::Clone(int) { return std::unique_ptr<Sampler>(new SobolSampler(*this)); }
int SobolSampler::DeviceSampler() const { return PBR_SAMPLER_SOBOL; }
Point2i SobolSampler::SampleRaster() const {
    return Point2i(sampleBounds.pMax.x - sampleBounds.pMin.x, sampleBounds.pMax.y - sampleBounds.pMin.y);
}

// ---- Sampler (Sampler/Sampler.cpp:7-67)
void Sampler::StartPixel(const Point2i& p) {
    currentPixel = p;
    currentPixelSampleIndex = 0;
    array1DOffset = array2DOffset = 0;
}
CameraSample Sampler::GetCameraSample(const Point2i& pRaster) {
    CameraSample cs;
    const Point2f u = Get2D();
    cs.pFilm = Point2f((float)pRaster.x + u.x, (float)pRaster.y + u.y);
    cs.time = Get1D();
    cs.pLens = Get2D();
    return cs;
}
bool Sampler::StartNextSample() {
    array1DOffset = array2DOffset = 0;
    return ++currentPixelSampleIndex < samplesPerPixel;
}
bool Sampler::SetSampleNumber(int64_t sampleNum) {
    array1DOffset = array2DOffset = 0;
    currentPixelSampleIndex = sampleNum;
    return currentPixelSampleIndex < samplesPerPixel;
}
void Sampler::Request1DArray(int n) {
    samples1DArraySizes.push_back(n);
    sampleArray1D.push_back(std::vector<float>((size_t)n * samplesPerPixel));
}
void Sampler::Request2DArray(int n) {
    samples2DArraySizes.push_back(n);
    sampleArray2D.push_back(std::vector<Point2f>((size_t)n * samplesPerPixel));
}
const float* Sampler::Get1DArray(int n) {
    if (array1DOffset == sampleArray1D.size()) return nullptr;
    return &sampleArray1D[array1DOffset++][currentPixelSampleIndex * n];
}
const Point2f* Sampler::Get2DArray(int n) {
    if (array2DOffset == sampleArray2D.size()) return nullptr;
    return &sampleArray2D[array2DOffset++][currentPixelSampleIndex * n];
}

// ---- PixelSampler (Sampler/Sampler.cpp:67-95)
PixelSampler::PixelSampler(int64_t samplesPerPixel, int nSampledDimensions) : Sampler(samplesPerPixel) {
    for (int i = 0; i < nSampledDimensions; ++i) {
        samples1D.push_back(std::vector<float>(samplesPerPixel));
        samples2D.push_back(std::vector<Point2f>(samplesPerPixel));
    }
}
bool PixelSampler::StartNextSample() {
    current1DDimension = current2DDimension = 0;
    return Sampler::StartNextSample();
}
bool PixelSampler::SetSampleNumber(int64_t sampleNum) {
    current1DDimension = current2DDimension = 0;
    return Sampler::SetSampleNumber(sampleNum);
}
float PixelSampler::Get1D() {
    if (current1DDimension < (int)samples1D.size()) return samples1D[current1DDimension++][currentPixelSampleIndex];
    return rng.UniformFloat();
}
Point2f PixelSampler::Get2D() {
    if (current2DDimension < (int)samples2D.size()) return samples2D[current2DDimension++][currentPixelSampleIndex];
    const float x = rng.UniformFloat(), y = rng.UniformFloat();   // Point2f(rng.UniformFloat(), rng.UniformFloat())
    return Point2f(x, y);
}

// ---- GlobalSampler (Sampler/Sampler.cpp:97-143)
void GlobalSampler::SampleDimensions(int64_t index, int firstDim, int n, float* out) const {
    for (int k = 0; k < n; ++k) out[k] = SampleDimension(index, firstDim + k);
}
void GlobalSampler::GetIndicesForSamples(int64_t firstSample, int n, int64_t* out) const {
    for (int k = 0; k < n; ++k) out[k] = GetIndexForSample(firstSample + k);
}
void GlobalSampler::SampleValues(const std::vector<int64_t>& sampleNums, const std::vector<int>& dims, float* out) const {
    if (sampleNums.size() != dims.size()) throw std::invalid_argument("SampleValues: sizes differ");
    for (size_t i = 0; i < dims.size(); ++i) SampleDimensions(GetIndexForSample(sampleNums[i]), dims[i], 1, &out[i]);
}
float GlobalSampler::SampleValue(int64_t sampleNum, int dim) const {
    float v = 0;
    SampleDimensions(GetIndexForSample(sampleNum), dim, 1, &v);
    return v;
}
void GlobalSampler::SampleDimensionsOf(const int64_t* index, int count, int firstDim, int n, float* out) const {
    for (int k = 0; k < count; ++k) SampleDimensions(index[k], firstDim, n, out + (size_t)k * n);
}
// GetIndexForSample is a pure function of the pixel and the sample number (Sampler.h:69), so the
// pixel's spp indices are fetched once, in StartPixel (one device query for the device samplers),
// and a sample's index is looked up when its first value is (the reference computes it in
// StartNextSample, including the unused one past the last sample).
int64_t GlobalSampler::indexOf(int64_t sampleNum) const {
    if (sampleNum >= 0 && sampleNum < (int64_t)pixelIndex.size()) return pixelIndex[(size_t)sampleNum];
    return GetIndexForSample(sampleNum);
}
int64_t GlobalSampler::CurrentIndex() const {
    if (!intervalKnown) {
        intervalSampleIndex = indexOf(intervalSample);
        intervalKnown = true;
    }
    return intervalSampleIndex;
}
// SampleDimension(intervalSampleIndex, dim) through a block cache: a device sampler answers the
// block with one query
float GlobalSampler::value(int dim) {
    if (cacheBase < 0 || dim < cacheBase || dim >= cacheBase + kValueBlock) {
        const int n = std::max(1, std::min(kValueBlock, MaxDimensions() - dim));
        SampleDimensions(CurrentIndex(), dim, n, cache);
        cacheBase = dim;
    }
    return cache[dim - cacheBase];
}
void GlobalSampler::StartPixel(const Point2i& p) {
    Sampler::StartPixel(p);
    dimension = 0;
    cacheBase = -1;
    pixelIndex.assign((size_t)samplesPerPixel, 0);
    GetIndicesForSamples(0, (int)samplesPerPixel, pixelIndex.data());
    intervalSample = 0;
    intervalKnown = false;
    arrayEndDim = arrayStartDim + (int)sampleArray1D.size() + 2 * (int)sampleArray2D.size();
    // the arrays of every sample of the pixel (Sampler.cpp:103-122): one batch per array
    for (size_t i = 0; i < samples1DArraySizes.size(); ++i) {
        const int nSamples = samples1DArraySizes[i] * (int)samplesPerPixel;
        std::vector<int64_t> idx(nSamples);
        GetIndicesForSamples(0, nSamples, idx.data());
        SampleDimensionsOf(idx.data(), nSamples, arrayStartDim + (int)i, 1, sampleArray1D[i].data());
    }
    int dim = arrayStartDim + (int)samples1DArraySizes.size();
    for (size_t i = 0; i < samples2DArraySizes.size(); ++i, dim += 2) {
        const int nSamples = samples2DArraySizes[i] * (int)samplesPerPixel;
        std::vector<int64_t> idx(nSamples);
        GetIndicesForSamples(0, nSamples, idx.data());
        std::vector<float> v(2 * (size_t)nSamples);
        SampleDimensionsOf(idx.data(), nSamples, dim, 2, v.data());
        for (int j = 0; j < nSamples; ++j) sampleArray2D[i][j] = Point2f(v[2 * j], v[2 * j + 1]);
    }
}
bool GlobalSampler::StartNextSample() {
    dimension = 0;
    cacheBase = -1;
    intervalSample = currentPixelSampleIndex + 1;
    intervalKnown = false;
    return Sampler::StartNextSample();
}
bool GlobalSampler::SetSampleNumber(int64_t sampleNum) {
    dimension = 0;
    cacheBase = -1;
    intervalSample = sampleNum;
    intervalKnown = false;
    return Sampler::SetSampleNumber(sampleNum);
}
float GlobalSampler::Get1D() {
    if (dimension >= arrayStartDim && dimension < arrayEndDim) dimension = arrayEndDim;
    return value(dimension++);
}
Point2f GlobalSampler::Get2D() {
    if (dimension + 1 >= arrayStartDim && dimension < arrayEndDim) dimension = arrayEndDim;
    const float x = value(dimension), y = value(dimension + 1);
    dimension += 2;
    return Point2f(x, y);
}

// ---- the device samplers' GetIndexForSample / SampleDimension (pbr_hip_sample_index /
// pbr_hip_sample_dimensions; Halton.cpp:61-92, pbrt-v3 SobolSampler)
namespace {
void device_indices(int type, Point2i raster, int64_t spp, const Point2i& pixel, int64_t first, int n, int64_t* out) {
    if (n <= 0) return;
    std::vector<int32_t> q(3 * (size_t)n);
    for (int k = 0; k < n; ++k) {
        if (first + k < 0 || first + k > 0x7fffffff) throw std::out_of_range("sample number beyond 31 bits");
        q[3 * k] = pixel.x; q[3 * k + 1] = pixel.y; q[3 * k + 2] = (int32_t)(first + k);
    }
    pbr_hip_ctx* h = helper_ctx();
    check(h, pbr_hip_sample_index(h, type, raster.x, raster.y, (int)spp, n, q.data(), out), "pbr_hip_sample_index");
}
void device_dimensions(int type, Point2i raster, const Point2i& pixel, int64_t index, int first, int n, int maxDims, float* out) {
    if (n <= 0) return;
    if (first < 0 || first + n > maxDims) throw std::out_of_range("sampler dimension beyond the sampler's tables");
    std::vector<int64_t> idx((size_t)n, index);
    std::vector<int32_t> q(3 * (size_t)n);
    for (int k = 0; k < n; ++k) { q[3 * k] = pixel.x; q[3 * k + 1] = pixel.y; q[3 * k + 2] = first + k; }
    pbr_hip_ctx* h = helper_ctx();
    check(h, pbr_hip_sample_dimensions(h, type, raster.x, raster.y, n, idx.data(), q.data(), out), "pbr_hip_sample_dimensions");
}
// dimensions [first, first + n) of `count` indices in one query (index-major)
void device_dimensions_of(int type, Point2i raster, const Point2i& pixel, const int64_t* index, int count, int first, int n,
                          int maxDims, float* out) {
    if (count <= 0 || n <= 0) return;
    if (first < 0 || first + n > maxDims) throw std::out_of_range("sampler dimension beyond the sampler's tables");
    const size_t m = (size_t)count * n;
    std::vector<int64_t> idx(m);
    std::vector<int32_t> q(3 * m);
    for (int k = 0; k < count; ++k)
        for (int d = 0; d < n; ++d) {
            const size_t e = (size_t)k * n + d;
            idx[e] = index[k];
            q[3 * e] = pixel.x; q[3 * e + 1] = pixel.y; q[3 * e + 2] = first + d;
        }
    pbr_hip_ctx* h = helper_ctx();
    check(h, pbr_hip_sample_dimensions(h, type, raster.x, raster.y, (int)m, idx.data(), q.data(), out), "pbr_hip_sample_dimensions");
}
}  // namespace
int64_t HaltonSampler::GetIndexForSample(int64_t sampleNum) const {
    int64_t v = 0;
    device_indices(PBR_SAMPLER_HALTON, SampleRaster(), samplesPerPixel, currentPixel, sampleNum, 1, &v);
    return v;
}
void HaltonSampler::GetIndicesForSamples(int64_t firstSample, int n, int64_t* out) const {
    device_indices(PBR_SAMPLER_HALTON, SampleRaster(), samplesPerPixel, currentPixel, firstSample, n, out);
}
float HaltonSampler::SampleDimension(int64_t index, int dimension) const {
    float v = 0;
    device_dimensions(PBR_SAMPLER_HALTON, SampleRaster(), currentPixel, index, dimension, 1, MaxDimensions(), &v);
    return v;
}
void HaltonSampler::SampleDimensions(int64_t index, int firstDim, int n, float* out) const {
    device_dimensions(PBR_SAMPLER_HALTON, SampleRaster(), currentPixel, index, firstDim, n, MaxDimensions(), out);
}
void HaltonSampler::SampleDimensionsOf(const int64_t* index, int count, int firstDim, int n, float* out) const {
    device_dimensions_of(PBR_SAMPLER_HALTON, SampleRaster(), currentPixel, index, count, firstDim, n, MaxDimensions(), out);
}
int64_t SobolSampler::GetIndexForSample(int64_t sampleNum) const {
    int64_t v = 0;
    device_indices(PBR_SAMPLER_SOBOL, SampleRaster(), samplesPerPixel, currentPixel, sampleNum, 1, &v);
    return v;
}
void SobolSampler::GetIndicesForSamples(int64_t firstSample, int n, int64_t* out) const {
    device_indices(PBR_SAMPLER_SOBOL, SampleRaster(), samplesPerPixel, currentPixel, firstSample, n, out);
}
float SobolSampler::SampleDimension(int64_t index, int dimension) const {
    float v = 0;
    device_dimensions(PBR_SAMPLER_SOBOL, SampleRaster(), currentPixel, index, dimension, 1, MaxDimensions(), &v);
    return v;
}
void SobolSampler::SampleDimensions(int64_t index, int firstDim, int n, float* out) const {
    device_dimensions(PBR_SAMPLER_SOBOL, SampleRaster(), currentPixel, index, firstDim, n, MaxDimensions(), out);
}
void SobolSampler::SampleDimensionsOf(const int64_t* index, int count, int firstDim, int n, float* out) const {
    device_dimensions_of(PBR_SAMPLER_SOBOL, SampleRaster(), currentPixel, index, count, firstDim, n, MaxDimensions(), out);
}

// ============================================================================ flattening
struct FlatScene {
    pbr_scene_desc desc{};
    std::vector<pbr_shape_desc> shapes;
    std::vector<pbr_material_desc> materials;
    std::vector<pbr_light_desc> lights;
    std::vector<pbr_medium_desc> media;
    std::vector<pbr_texture_desc> textures;
    std::map<const void*, int> textureIndex;                 // ImageTexture → index (shared textures once)
    std::vector<std::vector<int32_t>> indexRuns;
    std::vector<std::shared_ptr<TriangleMesh>> meshes;   // keep P/N/UV alive
    std::vector<std::shared_ptr<SkyBoxLight>> skies;     // keep env data alive
    std::vector<std::shared_ptr<InfiniteAreaLight>> infs;
    std::map<const Medium*, int> mediumIndex;
};

namespace {
Spectrum spec(const SpectrumTexture& t, const char* what) {
    if (!t) throw std::invalid_argument(std::string("material texture missing: ") + what);
    return t->ConstantValue();
}
float flt(const FloatTexture& t, const char* what) {
    if (!t) throw std::invalid_argument(std::string("material texture missing: ") + what);
    return t->ConstantValue();
}
void put(float* d, const Spectrum& s) { d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; }

// An image texture in a material slot: registered once per scene, referenced as index + 1.
template <typename T>
const ImageTextureData* image_of(const std::shared_ptr<Texture<T>>& t) {
    if (auto* a = dynamic_cast<const ImageTexture<RGBSpectrum, Spectrum>*>(t.get())) return &a->Image();
    if (auto* b = dynamic_cast<const ImageTexture<float, float>*>(t.get())) return &b->Image();
    return nullptr;
}
int texture_slot(FlatScene* F, const ImageTextureData* im) {
    auto it = F->textureIndex.find(im);
    if (it != F->textureIndex.end()) return it->second + 1;
    if (!im->mapping) throw std::invalid_argument("ImageTexture: only UVMapping2D is on the GPU path");
    pbr_texture_desc t;
    std::memset(&t, 0, sizeof(t));
    t.is_float = im->isFloat;
    t.width = im->width; t.height = im->height; t.components = im->components;
    t.data = im->data.empty() ? nullptr : im->data.data();
    t.scale = im->scale; t.gamma = im->gamma; t.wrap = (int)im->wrapMode;
    t.trilinear = im->doTrilinear; t.max_aniso = im->maxAniso;
    t.su = im->mapping->su; t.sv = im->mapping->sv; t.du = im->mapping->du; t.dv = im->mapping->dv;
    F->textureIndex[im] = (int)F->textures.size();
    F->textures.push_back(t);
    return (int)F->textures.size();
}

pbr_material_desc material_desc(FlatScene* F, const Material* m) {
    pbr_material_desc d;
    std::memset(&d, 0, sizeof(d));
    // a slot holding an ImageTexture is flattened as a texture reference, else as its constant
    auto sl = [&](const SpectrumTexture& t, int slot, float* out, const char* what) {
        if (const ImageTextureData* im = image_of(t)) d.tex[slot] = texture_slot(F, im);
        else put(out, spec(t, what));
    };
    auto fl = [&](const FloatTexture& t, int slot, float* out, const char* what) {
        if (const ImageTextureData* im = image_of(t)) d.tex[slot] = texture_slot(F, im);
        else *out = flt(t, what);
    };
    if (auto* x = dynamic_cast<const MatteMaterial*>(m)) {
        d.type = PBR_MAT_MATTE;
        sl(x->Kd, PBR_TEX_KD, d.Kd, "Kd");
        fl(x->sigma, PBR_TEX_SIGMA, &d.sigma, "sigma");
    } else if (auto* x = dynamic_cast<const MirrorMaterial*>(m)) {
        d.type = PBR_MAT_MIRROR;
        sl(x->Kr, PBR_TEX_KR, d.Kr, "Kr");
    } else if (auto* x = dynamic_cast<const GlassMaterial*>(m)) {
        d.type = PBR_MAT_GLASS;
        sl(x->Kr, PBR_TEX_KR, d.Kr, "Kr");
        sl(x->Kt, PBR_TEX_KT, d.Kt, "Kt");
        d.uroughness = flt(x->uRoughness, "uRoughness");
        d.vroughness = flt(x->vRoughness, "vRoughness");
        d.eta = flt(x->index, "index");
        d.remap_roughness = x->remapRoughness;
    } else if (auto* x = dynamic_cast<const MetalMaterial*>(m)) {
        d.type = PBR_MAT_METAL;
        put(d.metal_eta, spec(x->eta, "eta"));
        put(d.metal_k, spec(x->k, "k"));
        d.roughness = x->roughness ? x->roughness->ConstantValue() : 0.f;
        d.has_uv_roughness = (x->uRoughness && x->vRoughness) ? 1 : 0;
        if (d.has_uv_roughness) { d.uroughness = x->uRoughness->ConstantValue(); d.vroughness = x->vRoughness->ConstantValue(); }
        else if (!x->roughness) throw std::invalid_argument("MetalMaterial: no roughness");
        d.remap_roughness = x->remapRoughness;
    } else if (auto* x = dynamic_cast<const PlasticMaterial*>(m)) {
        d.type = PBR_MAT_PLASTIC;
        sl(x->Kd, PBR_TEX_KD, d.Kd, "Kd");
        sl(x->Ks, PBR_TEX_KS, d.Ks, "Ks");
        fl(x->roughness, PBR_TEX_ROUGHNESS, &d.roughness, "roughness");
        d.remap_roughness = x->remapRoughness;
    } else {
        throw std::invalid_argument("material type not on the GPU path");
    }
    return d;
}
}  // namespace

int MediumIndex(const FlatScene& f, const Medium* m) {
    if (!m) return -1;
    auto it = f.mediumIndex.find(m);
    if (it == f.mediumIndex.end()) throw std::invalid_argument("medium not part of the scene");
    return it->second;
}

std::shared_ptr<FlatScene> FlattenScene(const Scene& scene, const Medium* cameraMedium) {
    auto F = std::make_shared<FlatScene>();
    auto* bvh = dynamic_cast<const BVHAccel*>(scene.GetAggregate().get());
    if (!bvh) throw std::invalid_argument("Scene aggregate must be a BVHAccel");
    const auto& prims = bvh->Primitives();
    // media
    auto addMedium = [&](const Medium* m) {
        if (!m || F->mediumIndex.count(m)) return;
        auto* h = dynamic_cast<const HomogeneousMedium*>(m);
        if (!h) throw std::invalid_argument("only HomogeneousMedium is on the GPU path");
        pbr_medium_desc d;
        put(d.sigma_a, h->sigma_a);
        put(d.sigma_s, h->sigma_s);
        d.g = h->g;
        F->mediumIndex[m] = (int)F->media.size();
        F->media.push_back(d);
    };
    std::vector<const GeometricPrimitive*> gps;
    gps.reserve(prims.size());
    for (const auto& p : prims) {
        auto* gp = dynamic_cast<const GeometricPrimitive*>(p.get());
        if (!gp) throw std::invalid_argument("BVHAccel primitives must be GeometricPrimitives");
        gps.push_back(gp);
        addMedium(gp->mediumInterface.inside);
        addMedium(gp->mediumInterface.outside);
    }
    for (const auto& l : scene.lights) { addMedium(l->mediumInterface.inside); addMedium(l->mediumInterface.outside); }
    addMedium(cameraMedium);
    // materials
    std::map<const Material*, int> matIndex;
    for (auto* gp : gps) {
        const Material* m = gp->material.get();
        if (!m || matIndex.count(m)) continue;
        matIndex[m] = (int)F->materials.size();
        F->materials.push_back(material_desc(F.get(), m));
    }
    // lights: scene.lights order; area lights are bound to their shape below
    std::unordered_map<const Light*, int> lightIndex;
    for (size_t i = 0; i < scene.lights.size(); ++i) lightIndex[scene.lights[i].get()] = (int)i;
    F->lights.resize(scene.lights.size());
    std::vector<bool> boundArea(scene.lights.size(), false);
    // shapes: maximal runs of consecutive triangles sharing mesh, transform, material, medium
    // interface and consecutively numbered area lights
    size_t i = 0;
    while (i < gps.size()) {
        const GeometricPrimitive* gp = gps[i];
        pbr_shape_desc sd;
        std::memset(&sd, 0, sizeof(sd));
        sd.material = gp->material ? matIndex[gp->material.get()] : -1;
        sd.medium_inside = MediumIndex(*F, gp->mediumInterface.inside);
        sd.medium_outside = MediumIndex(*F, gp->mediumInterface.outside);
        sd.reverse_orientation = gp->shape->reverseOrientation;
        auto lightOf = [&](const GeometricPrimitive* g) -> int {
            if (!g->areaLight) return -1;
            auto it = lightIndex.find(g->areaLight.get());
            if (it == lightIndex.end()) throw std::invalid_argument("area light is not in Scene::lights");
            return it->second;
        };
        const int firstLight = lightOf(gp);
        const int shapeIdx = (int)F->shapes.size();
        if (auto* tri = dynamic_cast<const Triangle*>(gp->shape.get())) {
            const auto& mesh = tri->mesh;
            std::vector<int32_t> idx;
            size_t j = i;
            while (j < gps.size()) {
                const GeometricPrimitive* g = gps[j];
                auto* t = dynamic_cast<const Triangle*>(g->shape.get());
                if (!t || t->mesh != mesh || t->reverseOrientation != tri->reverseOrientation || g->material != gp->material ||
                    g->mediumInterface.inside != gp->mediumInterface.inside ||
                    g->mediumInterface.outside != gp->mediumInterface.outside)
                    break;
                int li = lightOf(g);
                int k = (int)(j - i);
                if ((firstLight < 0) != (li < 0) || (firstLight >= 0 && li != firstLight + k)) break;
                if (li >= 0) {
                    auto* dl = dynamic_cast<const DiffuseAreaLight*>(g->areaLight.get());
                    if (!dl || dl->shape.get() != g->shape.get()) throw std::invalid_argument("area light shape mismatch");
                    pbr_light_desc& L = F->lights[li];
                    std::memset(&L, 0, sizeof(L));
                    L.type = PBR_LIGHT_DIFFUSE_AREA;
                    fill_transform(dl->LightToWorld, &L.light_to_world);
                    put(L.Le, dl->Lemit);
                    L.shape = shapeIdx;
                    L.triangle = k;
                    L.two_sided = dl->twoSided;
                    L.n_samples = dl->nSamples;
                    L.medium_inside = MediumIndex(*F, dl->mediumInterface.inside);
                    L.medium_outside = MediumIndex(*F, dl->mediumInterface.outside);
                    boundArea[li] = true;
                }
                const int* v = &mesh->vertexIndices[(size_t)3 * t->triNumber];
                idx.insert(idx.end(), v, v + 3);
                ++j;
            }
            sd.type = PBR_SHAPE_TRIANGLE_MESH;
            fill_transform(mesh->objectToWorld, &sd.object_to_world);
            sd.n_triangles = (int)(j - i);
            sd.n_vertices = mesh->nVertices;
            F->indexRuns.push_back(std::move(idx));
            sd.indices = F->indexRuns.back().data();
            sd.P = mesh->p.data();
            sd.N = mesh->n.empty() ? nullptr : mesh->n.data();
            sd.UV = mesh->uv.empty() ? nullptr : mesh->uv.data();
            sd.area_light_first = firstLight;
            F->meshes.push_back(mesh);
            i = j;
        } else if (auto* sph = dynamic_cast<const Sphere*>(gp->shape.get())) {
            if (firstLight >= 0) throw std::invalid_argument("sphere area lights are not on the GPU path");
            sd.type = PBR_SHAPE_SPHERE;
            fill_transform(*sph->ObjectToWorld, &sd.object_to_world);
            sd.radius = sph->radius;
            sd.area_light_first = -1;
            ++i;
        } else {
            throw std::invalid_argument("shape type not on the GPU path");
        }
        F->shapes.push_back(sd);
    }
    // index runs were moved into a growing vector: re-point after all insertions
    for (size_t s = 0, r = 0; s < F->shapes.size(); ++s)
        if (F->shapes[s].type == PBR_SHAPE_TRIANGLE_MESH) F->shapes[s].indices = F->indexRuns[r++].data();
    for (size_t li = 0; li < scene.lights.size(); ++li) {
        const Light* l = scene.lights[li].get();
        pbr_light_desc& L = F->lights[li];
        if (auto* pl = dynamic_cast<const PointLight*>(l)) {
            std::memset(&L, 0, sizeof(L));
            L.type = PBR_LIGHT_POINT;
            fill_transform(pl->LightToWorld, &L.light_to_world);
            put(L.I, pl->I);
            L.n_samples = pl->nSamples;
            L.medium_inside = MediumIndex(*F, pl->mediumInterface.inside);
            L.medium_outside = MediumIndex(*F, pl->mediumInterface.outside);
        } else if (auto* sk = dynamic_cast<const SkyBoxLight*>(l)) {
            std::memset(&L, 0, sizeof(L));
            L.type = PBR_LIGHT_SKYBOX;
            fill_transform(sk->LightToWorld, &L.light_to_world);
            L.world_center[0] = sk->worldCenter.x; L.world_center[1] = sk->worldCenter.y; L.world_center[2] = sk->worldCenter.z;
            L.world_radius = sk->worldRadius;
            L.env_width = sk->imageWidth;
            L.env_height = sk->imageHeight;
            L.env_components = sk->nrComponents;
            L.env_data = sk->data.empty() ? nullptr : sk->data.data();
            L.n_samples = sk->nSamples;
            L.medium_inside = L.medium_outside = -1;
            F->skies.push_back(std::static_pointer_cast<SkyBoxLight>(scene.lights[li]));
        } else if (auto* il = dynamic_cast<const InfiniteAreaLight*>(l)) {
            std::memset(&L, 0, sizeof(L));
            L.type = PBR_LIGHT_INFINITE_AREA;
            fill_transform(il->LightToWorld, &L.light_to_world);
            put(L.Le, il->L);
            L.env_width = il->imageWidth;
            L.env_height = il->imageHeight;
            L.env_components = il->nrComponents;
            L.env_data = il->data.empty() ? nullptr : il->data.data();
            L.n_samples = il->nSamples;
            L.medium_inside = L.medium_outside = -1;
            F->infs.push_back(std::static_pointer_cast<InfiniteAreaLight>(scene.lights[li]));
        } else if (dynamic_cast<const DiffuseAreaLight*>(l)) {
            if (!boundArea[li]) throw std::invalid_argument("DiffuseAreaLight whose shape is not a scene triangle");
        } else {
            throw std::invalid_argument("light type not on the GPU path");
        }
    }
    pbr_scene_desc& d = F->desc;
    d.abi_version = PBR_HIP_ABI_VERSION;
    d.n_shapes = (int)F->shapes.size();
    d.shapes = F->shapes.data();
    d.n_materials = (int)F->materials.size();
    d.materials = F->materials.data();
    d.n_lights = (int)F->lights.size();
    d.lights = F->lights.data();
    d.n_media = (int)F->media.size();
    d.media = F->media.data();
    d.max_prims_in_node = bvh->maxPrimsInNode;
    d.split_method = (int)bvh->splitMethod;   // SAH, HLBVH, Middle, EqualCounts = pbr_split_method
    d.n_textures = (int)F->textures.size();
    d.textures = F->textures.data();
    return F;
}

const pbr_scene_desc* SceneDesc(const FlatScene& f) { return &f.desc; }

// ============================================================================ integrators
SamplerIntegrator::SamplerIntegrator(std::shared_ptr<const Camera> camera, std::shared_ptr<Sampler> sampler,
                                     const Bounds2i& pixelBounds, FrameBuffer* m_FrameBuffer)
    : camera(std::move(camera)), sampler(std::move(sampler)), pixelBounds(pixelBounds), m_FrameBuffer(m_FrameBuffer) {}

SamplerIntegrator::~SamplerIntegrator() {
    if (ctx) pbr_hip_destroy(ctx);
}

int WhittedIntegrator::IntegratorType() const { return PBR_INTEGRATOR_WHITTED; }
int PathIntegrator::IntegratorType() const { return PBR_INTEGRATOR_PATH; }
int VolPathIntegrator::IntegratorType() const { return PBR_INTEGRATOR_VOLPATH; }
int PathIntegrator::LightStrategy() const {
    // LightDistrib.cpp:10-21: "uniform" and "power"; "spatial" (the default) falls back to uniform
    return lightSampleStrategy == "power" ? PBR_LIGHTS_POWER : PBR_LIGHTS_UNIFORM;
}

namespace {
void check(pbr_hip_ctx* ctx, int rc, const char* what) {
    if (rc == PBR_OK) return;
    std::string msg = std::string(what) + " failed (" + std::to_string(rc) + ")";
    if (ctx) msg += ": " + std::string(pbr_hip_last_error(ctx));
    throw std::runtime_error(msg);
}
// The sample-table path (a GlobalSampler subclass the device cannot compute) holds the whole frame's
// values in host and device memory: up to this many bytes.
constexpr double kMaxSampleTableBytes = 16e9;
void camera_desc(const PerspectiveCamera& cam, pbr_camera_desc* c) {
    std::memset(c, 0, sizeof(*c));
    c->width = cam.RasterWidth;
    c->height = cam.RasterHeight;
    fill_transform(cam.CameraToWorld, &c->camera_to_world);
    c->fov = cam.fov;
    c->lens_radius = cam.lensRadius;
    c->focal_distance = cam.focalDistance;
    c->medium = -1;
    // A screen window other than CreatePerspectiveCamera's (Perspective.cpp:84-104): the camera's own
    // RasterToCamera, as ProjectiveCamera's constructor forms it (Camera.h:36-53), goes over instead.
    const float frame = (float)cam.RasterWidth / (float)cam.RasterHeight;
    const float sx = frame > 1.f ? frame : 1.f, sy = frame > 1.f ? 1.f : 1.f / frame;
    const Bounds2f& w = cam.screenWindow;
    if (w.pMin.x != -sx || w.pMax.x != sx || w.pMin.y != -sy || w.pMax.y != sy) {
        using namespace pbr::xform;
        const Xf camToScreen = perspective(cam.fov, 1e-2f, 1000.f);
        const Xf screenToRaster = compose(compose(scale((float)cam.RasterWidth, (float)cam.RasterHeight, 1),
                                                  scale(1 / (w.pMax.x - w.pMin.x), 1 / (w.pMin.y - w.pMax.y), 1)),
                                          translate(pbr::mk(-w.pMin.x, -w.pMax.y, 0)));
        const Xf r2c = compose(inverse(camToScreen), inverse(screenToRaster));
        c->use_raster_to_camera = 1;
        std::memcpy(c->raster_to_camera.m, &r2c.m.a[0][0], 64);
        std::memcpy(c->raster_to_camera.m_inv, &r2c.mi.a[0][0], 64);
    }
}
// The samplers the device runs: HaltonSampler (any raster: its values depend on the pixel only) and
// SobolSampler, whose resolution must be the camera's raster (the device derives it from there).
void check_sampler(const Sampler& s, const PerspectiveCamera& cam, const char* who) {
    const bool device = dynamic_cast<const HaltonSampler*>(&s) || dynamic_cast<const SobolSampler*>(&s);
    if (!device && (s.DeviceSampler() != PBR_SAMPLER_TABLE || !dynamic_cast<const GlobalSampler*>(&s)))
        throw std::invalid_argument(std::string(who) + ": HaltonSampler, SobolSampler or a GlobalSampler subclass "
                                                       "(PixelSampler's separate 1D / 2D streams are not on the GPU path)");
    if (s.DeviceSampler() == PBR_SAMPLER_SOBOL && (s.SampleRaster().x != cam.RasterWidth || s.SampleRaster().y != cam.RasterHeight))
        throw std::invalid_argument(std::string(who) + ": SobolSampler bounds must be the camera raster");
}
// Device 0 context for the stateless helpers (camera rays, sampler values).  Kept for the life of the
// process: destroying it from a static destructor could run after the HIP runtime has shut down.
pbr_hip_ctx* helper_ctx() {
    static pbr_hip_ctx* h = nullptr;
    if (!h) check(nullptr, pbr_hip_create(0, &h), "pbr_hip_create");
    return h;
}
}  // namespace

void SamplerIntegrator::Render(const Scene& scene, double& timeConsume) {
    if (!devices.empty()) return RenderMulti(scene, timeConsume);
    auto t0 = std::chrono::steady_clock::now();
    auto* cam = dynamic_cast<const PerspectiveCamera*>(camera.get());
    if (!cam) throw std::invalid_argument("Render: only PerspectiveCamera is on the GPU path");
    check_sampler(*sampler, *cam, "Render");
    const int W = pixelBounds.pMax.x, H = pixelBounds.pMax.y;   // the reference reads pMax only
    if (W <= 0 || H <= 0 || W > cam->RasterWidth || H > cam->RasterHeight)
        throw std::invalid_argument("Render: pixelBounds outside the camera raster");
    ensure_scene(scene);
    auto flat = FlattenScene(scene, cam->medium);   // for the camera medium's index
    pbr_render_desc rd;
    std::memset(&rd, 0, sizeof(rd));
    rd.integrator = IntegratorType();
    rd.max_depth = MaxDepth();
    rd.rr_threshold = RRThreshold();
    rd.light_strategy = LightStrategy();
    rd.sampler = sampler->DeviceSampler();
    rd.spp = (int)sampler->samplesPerPixel;
    camera_desc(*cam, &rd.camera);
    rd.camera.medium = MediumIndex(*flat, cam->medium);
    std::vector<pbr_tile> tl;
    if (!tiles.empty()) {
        for (const Bounds2i& b : tiles) tl.push_back({b.pMin.x, b.pMin.y, b.pMax.x, b.pMax.y});
    } else {
        tl.push_back({0, 0, W, H});
    }
    std::vector<float> table;
    // A GlobalSampler the device cannot compute: its values for every pixel and sample of the frame,
    // taken the way Render's loop takes them (Integrator.cpp:290-300: Clone(offset), StartPixel, then
    // sample after sample), for `dims` dimensions.
    auto tabulate = [&](int dims) {
        const int Wr = cam->RasterWidth, Hr = cam->RasterHeight, spp = rd.spp;
        const double bytes = (double)Wr * Hr * spp * dims * sizeof(float);
        if (bytes > kMaxSampleTableBytes)
            throw std::invalid_argument("Render: a " + std::to_string((int)(bytes / 1e9)) + " GB sample table for this " +
                                        "GlobalSampler is beyond the " + std::to_string((int)(kMaxSampleTableBytes / 1e9)) +
                                        " GB the sample-table path takes (fewer samples per pixel or a smaller frame)");
        table.assign((size_t)Wr * Hr * spp * dims, 0.f);
        for (const pbr_tile& t : tl)
            for (int y = t.y0; y < t.y1; ++y)
                for (int x = t.x0; x < t.x1; ++x) {
                    std::unique_ptr<Sampler> ps = sampler->Clone(pixelBounds.pMax.x * y + x);
                    auto* g = dynamic_cast<GlobalSampler*>(ps.get());
                    if (!g) throw std::invalid_argument("Render: Clone of a GlobalSampler must be a GlobalSampler");
                    g->StartPixel(Point2i(x, y));
                    for (int k = 0; k < spp; ++k) {
                        if (k > 0) g->StartNextSample();
                        g->SampleDimensions(g->CurrentIndex(), 0, dims, &table[(((size_t)y * Wr + x) * spp + k) * dims]);
                    }
                }
        rd.sample_table = table.data();
        rd.table_dims = dims;
    };
    int dims = 0;
    if (rd.sampler == PBR_SAMPLER_TABLE) {
        // The dimensions the integrator reaches: 5 camera dimensions, then per bounce at most 2 per
        // light + 2 (Whitted), 8 (Path: light choice, light and BSDF samples, its own BSDF sample,
        // roulette) or 10 (VolPath: + medium sampling).  A VolPath path also draws HomogeneousMedium::
        // Sample's 2 dimensions at each material-less boundary it crosses inside a medium, which does
        // not count as a bounce (VolPathIntegrator.cpp:68-71): when a path asks the table for more
        // than it holds (the device's kGuardSampleTable), the frame is tabulated again with twice the
        // dimensions and rendered again, below.
        const int depth = std::max(1, MaxDepth()), nl = (int)scene.lights.size();
        dims = IntegratorType() == PBR_INTEGRATOR_WHITTED ? 5 + depth * (2 * std::max(1, nl) + 2) + 2
               : IntegratorType() == PBR_INTEGRATOR_PATH ? 5 + (depth + 1) * 8 + 2
                                                         : 5 + (depth + 1) * 10 + 2;
        tabulate(dims);
    }
    rd.n_tiles = (int)tl.size();
    rd.tiles = tl.data();
    size_t npx = 0;
    for (const pbr_tile& t : tl) npx += (size_t)(t.x1 - t.x0) * (t.y1 - t.y0);
    std::vector<float> rgb(npx * 3);
    std::vector<uint8_t> rgba(npx * 4);
    pbr_render_stats st;
    // Retry only when the sample-table bound is the ONE guard bit the frame tripped (check_guard lists
    // the bits in a fixed order and the sample table's comes last, so its clause then opens the
    // message), at most kMaxTableRetries times; any other failure — or a table that would outgrow
    // kMaxSampleTableBytes — reports the render's original error.
    static const char kTableOnly[] = "a path asked the sample table for a dimension beyond table_dims; ";
    constexpr int kMaxTableRetries = 4;
    for (int retry = 0;; ++retry) {
        const int rc = pbr_hip_render(ctx, &rd, rgb.data(), rgba.data(), &st);
        if (rc == PBR_E_UNSUPPORTED && rd.sampler == PBR_SAMPLER_TABLE && retry < kMaxTableRetries &&
            std::strncmp(pbr_hip_last_error(ctx), kTableOnly, sizeof(kTableOnly) - 1) == 0) {
            const std::string original = pbr_hip_last_error(ctx);
            dims *= 2;   // a path went past the table (medium boundaries): more dimensions, same frame
            try {
                tabulate(dims);
            } catch (const std::invalid_argument&) {
                throw std::runtime_error(std::string("pbr_hip_render: ") + original);
            }
            continue;
        }
        check(ctx, rc, "pbr_hip_render");
        break;
    }
    if (m_FrameBuffer) {
        if (m_FrameBuffer->width != W || m_FrameBuffer->height != H || m_FrameBuffer->channals < 3)
            throw std::invalid_argument("Render: FrameBuffer not initialised to the pixel bounds");
        size_t k = 0;
        for (const pbr_tile& t : tl)
            for (int y = t.y0; y < t.y1; ++y)
                for (int x = t.x0; x < t.x1; ++x, ++k)
                    for (int ch = 0; ch < m_FrameBuffer->channals; ++ch) {
                        // Integrator.cpp:341-344: set_uc(x, pMax.y - y - 1, ...) — the image is flipped
                        m_FrameBuffer->set_uc(x, H - y - 1, ch, rgba[4 * k + ch]);
                        m_FrameBuffer->set_fc(x, H - y - 1, ch, ch < 3 ? rgb[3 * k + ch] : 1.f);
                    }
    }
    stats.seconds = st.seconds;
    stats.kernel_ms = st.kernel_ms;
    stats.samples = st.samples;
    timeConsume = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    IntegratorRenderTime = (float)timeConsume;
}

// ============================================================================ scene queries
SceneDevice& Scene::device() const {
    if (dev) return *dev;
    auto d = std::make_unique<SceneDevice>();
    auto* bvh = dynamic_cast<const BVHAccel*>(aggregate.get());
    if (!bvh) throw std::invalid_argument("Scene queries need a BVHAccel aggregate");
    for (const auto& p : bvh->Primitives()) d->prims.push_back(p.get());
    d->flat = FlattenScene(*this, nullptr);
    check(nullptr, pbr_hip_create(queryDevice, &d->ctx), "pbr_hip_create");
    check(d->ctx, pbr_hip_upload_scene(d->ctx, SceneDesc(*d->flat)), "pbr_hip_upload_scene");
    float b[6];
    check(d->ctx, pbr_hip_bounds(d->ctx, -1, b), "pbr_hip_bounds");
    d->worldBound = Bounds3f(Point3f(b[0], b[1], b[2]), Point3f(b[3], b[4], b[5]));
    dev = std::move(d);
    return *dev;
}

const Bounds3f& Scene::WorldBound() const { return device().worldBound; }

namespace {
void ray_floats(const Ray& r, float* o) {
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z; o[3] = r.d.x; o[4] = r.d.y; o[5] = r.d.z; o[6] = r.tMax;
}
const Medium* medium_at(const FlatScene& f, int index) {
    if (index < 0) return nullptr;
    for (const auto& kv : f.mediumIndex)
        if (kv.second == index) return kv.first;
    return nullptr;
}
// GeometricPrimitive::Intersect's bookkeeping (Primitive.cpp:22-36): r.tMax = tHit, the
// interaction's primitive and medium interface
void fill_isect(const SceneDevice& d, const pbr_surface_hit& h, const Ray& r, SurfaceInteraction* si) {
    r.tMax = h.t;
    if (!si) return;
    si->p = Point3f(h.p[0], h.p[1], h.p[2]);
    si->pError = Vector3f(h.p_error[0], h.p_error[1], h.p_error[2]);
    si->wo = Vector3f(h.wo[0], h.wo[1], h.wo[2]);
    si->n = Normal3f(h.n[0], h.n[1], h.n[2]);
    si->shading.n = Normal3f(h.ns[0], h.ns[1], h.ns[2]);
    si->dpdu = si->shading.dpdu = Vector3f(h.dpdu[0], h.dpdu[1], h.dpdu[2]);
    si->uv = Point2f(h.uv[0], h.uv[1]);
    si->time = r.time;
    si->b0 = h.b[0]; si->b1 = h.b[1]; si->b2 = h.b[2];
    si->primIndex = h.prim;
    si->primitive = h.prim >= 0 && h.prim < (int)d.prims.size() ? d.prims[h.prim] : nullptr;
    const Medium* in = medium_at(*d.flat, h.medium_inside);
    const Medium* out = medium_at(*d.flat, h.medium_outside);
    si->mediumInterface = in != out ? MediumInterface(in, out) : MediumInterface(r.medium);
    si->bsdfMaterial = nullptr;
}
}  // namespace

void Scene::Intersect(const std::vector<Ray>& rays, std::vector<SurfaceInteraction>* isects, std::vector<char>* hit) const {
    SceneDevice& d = device();
    std::vector<float> rf(rays.size() * 7);
    for (size_t i = 0; i < rays.size(); ++i) ray_floats(rays[i], &rf[7 * i]);
    std::vector<pbr_surface_hit> out(rays.size());
    check(d.ctx, pbr_hip_query(d.ctx, (int)rays.size(), rf.data(), 0, -1, out.data()), "pbr_hip_query");
    if (isects) isects->assign(rays.size(), SurfaceInteraction());
    if (hit) hit->assign(rays.size(), 0);
    for (size_t i = 0; i < rays.size(); ++i) {
        if (hit) (*hit)[i] = (char)out[i].hit;
        if (out[i].hit) fill_isect(d, out[i], rays[i], isects ? &(*isects)[i] : nullptr);
    }
}

void Scene::IntersectP(const std::vector<Ray>& rays, std::vector<char>* hit) const {
    SceneDevice& d = device();
    std::vector<float> rf(rays.size() * 7);
    for (size_t i = 0; i < rays.size(); ++i) ray_floats(rays[i], &rf[7 * i]);
    std::vector<pbr_surface_hit> out(rays.size());
    check(d.ctx, pbr_hip_query(d.ctx, (int)rays.size(), rf.data(), 1, -1, out.data()), "pbr_hip_query");
    hit->assign(rays.size(), 0);
    for (size_t i = 0; i < rays.size(); ++i) (*hit)[i] = (char)out[i].hit;
}

bool Scene::Intersect(const Ray& ray, SurfaceInteraction* isect) const {   // Scene.cpp:20-24
    SceneDevice& d = device();
    float rf[7];
    ray_floats(ray, rf);
    pbr_surface_hit h;
    check(d.ctx, pbr_hip_query(d.ctx, 1, rf, 0, -1, &h), "pbr_hip_query");
    if (!h.hit) return false;
    fill_isect(d, h, ray, isect);
    return true;
}

bool Scene::IntersectP(const Ray& ray) const {   // Scene.cpp:26-28
    std::vector<char> hit;
    IntersectP(std::vector<Ray>{ray}, &hit);
    return hit[0] != 0;
}

bool Scene::IntersectPrimitive(int index, const Ray& ray, SurfaceInteraction* isect) const {
    SceneDevice& d = device();
    float rf[7];
    ray_floats(ray, rf);
    pbr_surface_hit h;
    check(d.ctx, pbr_hip_query(d.ctx, 1, rf, 0, index, &h), "pbr_hip_query");
    if (!h.hit) return false;
    fill_isect(d, h, ray, isect);
    return true;
}

bool Scene::IntersectPPrimitive(int index, const Ray& ray) const {
    SceneDevice& d = device();
    float rf[7];
    ray_floats(ray, rf);
    pbr_surface_hit h;
    check(d.ctx, pbr_hip_query(d.ctx, 1, rf, 1, index, &h), "pbr_hip_query");
    return h.hit != 0;
}

Bounds3f Scene::PrimitiveBound(int index) const {
    SceneDevice& d = device();
    float b[6];
    check(d.ctx, pbr_hip_bounds(d.ctx, index, b), "pbr_hip_bounds");
    return Bounds3f(Point3f(b[0], b[1], b[2]), Point3f(b[3], b[4], b[5]));
}

namespace {
const Scene& owner_of(const Scene* s, const char* what) {
    if (!s) throw std::logic_error(std::string(what) + ": the primitive belongs to no Scene (queries run on its device)");
    return *s;
}
}  // namespace

Bounds3f GeometricPrimitive::WorldBound() const { return owner_of(owner, "GeometricPrimitive::WorldBound").PrimitiveBound(ownerIndex); }
bool GeometricPrimitive::Intersect(const Ray& r, SurfaceInteraction* isect) const {
    return owner_of(owner, "GeometricPrimitive::Intersect").IntersectPrimitive(ownerIndex, r, isect);
}
bool GeometricPrimitive::IntersectP(const Ray& r) const {
    return owner_of(owner, "GeometricPrimitive::IntersectP").IntersectPPrimitive(ownerIndex, r);
}
void GeometricPrimitive::ComputeScatteringFunctions(SurfaceInteraction* isect, TransportMode mode, bool allowMultipleLobes) const {
    // Primitive.cpp:46-53: the material builds the BSDF; here the BSDF lives on the device, so the
    // interaction records which material scatters and how
    isect->bsdfMaterial = material.get();
    isect->mode = mode;
    isect->allowMultipleLobes = allowMultipleLobes;
}
Bounds3f BVHAccel::WorldBound() const { return owner_of(owner, "BVHAccel::WorldBound").WorldBound(); }
bool BVHAccel::Intersect(const Ray& r, SurfaceInteraction* isect) const {
    return owner_of(owner, "BVHAccel::Intersect").Intersect(r, isect);
}
bool BVHAccel::IntersectP(const Ray& r) const { return owner_of(owner, "BVHAccel::IntersectP").IntersectP(r); }

// ============================================================================ camera, sampler, Li
float PerspectiveCamera::GenerateRay(const CameraSample& sample, Ray* ray) const {   // Perspective.cpp:44-62
    if (lensRadius > 0) throw std::invalid_argument("PerspectiveCamera::GenerateRay: thin-lens cameras are not on the GPU path");
    pbr_camera_desc c;
    camera_desc(*this, &c);
    const float pf[2] = {sample.pFilm.x, sample.pFilm.y};
    float out[6];
    pbr_hip_ctx* h = helper_ctx();
    check(h, pbr_hip_camera_rays(h, &c, 1, pf, out), "pbr_hip_camera_rays");
    *ray = Ray(Point3f(out[0], out[1], out[2]), Vector3f(out[3], out[4], out[5]));
    ray->time = sample.time;
    ray->medium = medium;
    return 1;
}

void SamplerIntegrator::ensure_scene(const Scene& scene) const {
    auto* cam = dynamic_cast<const PerspectiveCamera*>(camera.get());
    const Medium* cm = cam ? cam->medium : nullptr;
    if (!ctx) check(nullptr, pbr_hip_create(device, &ctx), "pbr_hip_create");
    if (uploadedScene != scene.Id() || uploadedCameraMedium != cm) {
        auto flat = FlattenScene(scene, cm);
        check(ctx, pbr_hip_upload_scene(ctx, SceneDesc(*flat)), "pbr_hip_upload_scene");
        uploadedScene = scene.Id();
        uploadedCameraMedium = cm;
    }
}

void SamplerIntegrator::Preprocess(const Scene& scene, Sampler&) { ensure_scene(scene); }

std::vector<Spectrum> SamplerIntegrator::Li(const std::vector<Ray>& rays, const std::vector<Point2i>& pixels,
                                            const std::vector<int64_t>& samples, int dimension, const Scene& scene,
                                            int depth) const {
    return LiWith(*sampler, rays, pixels, samples, dimension, scene, depth);
}
std::vector<Spectrum> SamplerIntegrator::LiWith(const Sampler& smp, const std::vector<Ray>& rays,
                                                const std::vector<Point2i>& pixels, const std::vector<int64_t>& samples,
                                                int dimension, const Scene& scene, int depth) const {
    if (pixels.size() != rays.size() || samples.size() != rays.size())
        throw std::invalid_argument("Li: rays, pixels and samples differ in length");
    if (smp.DeviceSampler() != PBR_SAMPLER_HALTON && smp.DeviceSampler() != PBR_SAMPLER_SOBOL)
        throw std::invalid_argument("Li: only HaltonSampler and SobolSampler continue a sample on the device "
                                    "(other samplers render through Render)");
    ensure_scene(scene);
    pbr_render_desc rd;
    std::memset(&rd, 0, sizeof(rd));
    rd.integrator = IntegratorType();
    rd.max_depth = MaxDepth();
    rd.rr_threshold = RRThreshold();
    rd.light_strategy = LightStrategy();
    rd.sampler = smp.DeviceSampler();
    rd.spp = (int)smp.samplesPerPixel;
    rd.camera.width = smp.SampleRaster().x;   // the sampler's raster
    rd.camera.height = smp.SampleRaster().y;
    rd.camera.fov = 90.f;
    rd.camera.camera_to_world.m[0] = rd.camera.camera_to_world.m[5] = rd.camera.camera_to_world.m[10] =
        rd.camera.camera_to_world.m[15] = 1.f;
    rd.camera.camera_to_world.m_inv[0] = rd.camera.camera_to_world.m_inv[5] = rd.camera.camera_to_world.m_inv[10] =
        rd.camera.camera_to_world.m_inv[15] = 1.f;
    rd.camera.medium = -1;
    std::vector<float> rf(rays.size() * 7);
    std::vector<int32_t> q(rays.size() * 4);
    for (size_t i = 0; i < rays.size(); ++i) {
        ray_floats(rays[i], &rf[7 * i]);
        q[4 * i] = pixels[i].x; q[4 * i + 1] = pixels[i].y; q[4 * i + 2] = (int32_t)samples[i]; q[4 * i + 3] = dimension;
    }
    std::vector<float> L(rays.size() * 3);
    check(ctx, pbr_hip_li(ctx, &rd, (int)rays.size(), rf.data(), q.data(), depth, L.data()), "pbr_hip_li");
    std::vector<Spectrum> out(rays.size());
    for (size_t i = 0; i < rays.size(); ++i) { out[i][0] = L[3 * i]; out[i][1] = L[3 * i + 1]; out[i][2] = L[3 * i + 2]; }
    return out;
}

Spectrum SamplerIntegrator::Li(const RayDifferential& ray, const Scene& scene, Sampler& s, int depth) const {
    return LiWith(s, std::vector<Ray>{ray}, std::vector<Point2i>{s.CurrentPixel()},
                  std::vector<int64_t>{s.CurrentSampleNumber()}, s.CurrentDimension(), scene, depth)[0];
}

// ============================================================================ multi-GPU
std::vector<Bounds2i> TileGrid(int width, int height, int tile) {
    std::vector<Bounds2i> t;
    for (int y = 0; y < height; y += tile)
        for (int x = 0; x < width; x += tile)
            t.emplace_back(Point2i(x, y), Point2i(std::min(x + tile, width), std::min(y + tile, height)));
    return t;
}
std::vector<Bounds2i> TilesForRank(int width, int height, int rank, int world, int tile) {
    std::vector<Bounds2i> all = TileGrid(width, height, tile), mine;
    for (size_t i = 0; i < all.size(); ++i)
        if ((int)(i % (size_t)world) == rank) mine.push_back(all[i]);
    return mine;
}
namespace {
template <class T>
void assemble(const std::vector<Bounds2i>& tiles, const T* packed, int ch, int width, T* frame) {
    size_t k = 0;
    for (const Bounds2i& t : tiles)
        for (int y = t.pMin.y; y < t.pMax.y; ++y)
            for (int x = t.pMin.x; x < t.pMax.x; ++x, ++k)
                std::memcpy(frame + ((size_t)y * width + x) * ch, packed + k * ch, sizeof(T) * ch);
}
void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void nccl_check(ncclResult_t e, const char* what) {
    if (e != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(e));
}
}  // namespace
void AssembleTiles(const std::vector<Bounds2i>& tiles, const uint8_t* packed, int ch, int width, uint8_t* frame) {
    assemble(tiles, packed, ch, width, frame);
}
void AssembleTiles(const std::vector<Bounds2i>& tiles, const float* packed, int ch, int width, float* frame) {
    assemble(tiles, packed, ch, width, frame);
}

struct SamplerIntegrator::MultiGPU {
    std::vector<int> devs;
    int W = 0, H = 0;
    std::vector<pbr_hip_ctx*> ctx;
    std::vector<hipStream_t> streams;
    std::vector<ncclComm_t> comms;          // one per rank when the devices are distinct
    std::vector<std::vector<Bounds2i>> tiles;
    std::vector<size_t> npx;
    size_t maxPx = 0;
    std::vector<void*> sendU8, sendF32;     // per rank, on its device: maxPx pixels
    void *recvU8 = nullptr, *recvF32 = nullptr;   // on the first device: world × maxPx pixels
    std::vector<uint64_t> uploaded;
    std::vector<const Medium*> uploadedMedium;
    ~MultiGPU() {
        for (size_t r = 0; r < ctx.size(); ++r) {
            (void)hipSetDevice(devs[r]);
            if (r < streams.size() && streams[r]) (void)hipStreamSynchronize(streams[r]);
            if (r < sendU8.size() && sendU8[r]) (void)hipFree(sendU8[r]);
            if (r < sendF32.size() && sendF32[r]) (void)hipFree(sendF32[r]);
        }
        for (ncclComm_t c : comms) (void)ncclCommDestroy(c);
        if (!devs.empty()) {
            (void)hipSetDevice(devs[0]);
            if (recvU8) (void)hipFree(recvU8);
            if (recvF32) (void)hipFree(recvF32);
        }
        for (size_t r = 0; r < ctx.size(); ++r) {
            if (ctx[r]) pbr_hip_destroy(ctx[r]);
            if (r < streams.size() && streams[r]) { (void)hipSetDevice(devs[r]); (void)hipStreamDestroy(streams[r]); }
        }
    }
};

void SamplerIntegrator::RenderMulti(const Scene& scene, double& timeConsume) {
    auto t0 = std::chrono::steady_clock::now();
    auto* cam = dynamic_cast<const PerspectiveCamera*>(camera.get());
    if (!cam) throw std::invalid_argument("Render: only PerspectiveCamera is on the GPU path");
    check_sampler(*sampler, *cam, "Render");
    if (sampler->DeviceSampler() == PBR_SAMPLER_TABLE)
        throw std::invalid_argument("Render on several devices: custom GlobalSamplers render on one device");
    if (!tiles.empty()) throw std::invalid_argument("Render: SetTiles and SetDevices are exclusive");
    const int W = pixelBounds.pMax.x, H = pixelBounds.pMax.y;
    if (W <= 0 || H <= 0 || W > cam->RasterWidth || H > cam->RasterHeight)
        throw std::invalid_argument("Render: pixelBounds outside the camera raster");
    if (!m_FrameBuffer || m_FrameBuffer->width != W || m_FrameBuffer->height != H || m_FrameBuffer->channals < 3)
        throw std::invalid_argument("Render: FrameBuffer not initialised to the pixel bounds");
    const int world = (int)devices.size();
    if (!multi || multi->devs != devices || multi->W != W || multi->H != H) {
        multi.reset();   // release the old set first
        auto m = std::make_shared<MultiGPU>();
        m->devs = devices;
        m->W = W;
        m->H = H;
        for (int r = 0; r < world; ++r) {
            pbr_hip_ctx* c = nullptr;
            check(nullptr, pbr_hip_create(devices[r], &c), "pbr_hip_create");
            m->ctx.push_back(c);
            m->tiles.push_back(TilesForRank(W, H, r, world));
            size_t n = 0;
            for (const Bounds2i& t : m->tiles.back()) n += (size_t)(t.pMax.x - t.pMin.x) * (t.pMax.y - t.pMin.y);
            m->npx.push_back(n);
            m->maxPx = std::max(m->maxPx, n);
        }
        m->uploaded.assign(world, 0);
        m->uploadedMedium.assign(world, nullptr);
        for (int r = 0; r < world; ++r) {
            hip_check(hipSetDevice(devices[r]), "hipSetDevice");
            hipStream_t st;
            hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
            m->streams.push_back(st);
            void *u = nullptr, *f = nullptr;
            hip_check(hipMalloc(&u, std::max<size_t>(1, m->maxPx) * 4), "hipMalloc");
            hip_check(hipMalloc(&f, std::max<size_t>(1, m->maxPx) * 12), "hipMalloc");
            m->sendU8.push_back(u);
            m->sendF32.push_back(f);
        }
        hip_check(hipSetDevice(devices[0]), "hipSetDevice");
        hip_check(hipMalloc(&m->recvU8, std::max<size_t>(1, m->maxPx) * 4 * world), "hipMalloc");
        hip_check(hipMalloc(&m->recvF32, std::max<size_t>(1, m->maxPx) * 12 * world), "hipMalloc");
        std::vector<int> sorted = devices;
        std::sort(sorted.begin(), sorted.end());
        if (std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end()) {   // distinct: one RCCL communicator
            m->comms.resize(world);
            nccl_check(ncclCommInitAll(m->comms.data(), world, devices.data()), "ncclCommInitAll");
        }
        multi = m;
    }
    MultiGPU& m = *multi;
    auto flat = FlattenScene(scene, cam->medium);
    pbr_render_desc rd;
    std::memset(&rd, 0, sizeof(rd));
    rd.integrator = IntegratorType();
    rd.max_depth = MaxDepth();
    rd.rr_threshold = RRThreshold();
    rd.light_strategy = LightStrategy();
    rd.sampler = sampler->DeviceSampler();
    rd.spp = (int)sampler->samplesPerPixel;
    camera_desc(*cam, &rd.camera);
    rd.camera.medium = MediumIndex(*flat, cam->medium);
    rd.outputs_on_device = 1;
    // every rank's frame is enqueued on its own stream (asynchronous: no stats, device outputs)
    std::vector<std::vector<pbr_tile>> tl(world);
    for (int r = 0; r < world; ++r) {
        if (m.uploaded[r] != scene.Id() || m.uploadedMedium[r] != cam->medium) {
            check(m.ctx[r], pbr_hip_upload_scene(m.ctx[r], SceneDesc(*flat)), "pbr_hip_upload_scene");
            m.uploaded[r] = scene.Id();
            m.uploadedMedium[r] = cam->medium;
        }
        for (const Bounds2i& b : m.tiles[r]) tl[r].push_back({b.pMin.x, b.pMin.y, b.pMax.x, b.pMax.y});
        if (tl[r].empty()) continue;   // more ranks than tiles
        pbr_render_desc rr = rd;
        rr.n_tiles = (int)tl[r].size();
        rr.tiles = tl[r].data();
        rr.stream = m.streams[r];
        check(m.ctx[r], pbr_hip_render(m.ctx[r], &rr, (float*)m.sendF32[r], (uint8_t*)m.sendU8[r], nullptr), "pbr_hip_render");
    }
    // the exchange: rank spans → the first device
    std::vector<uint8_t> u8((size_t)world * m.maxPx * 4);
    std::vector<float> f32((size_t)world * m.maxPx * 3);
    if (!m.comms.empty()) {
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        for (int r = 0; r < world; ++r) {
            nccl_check(ncclGather(m.sendU8[r], r == 0 ? m.recvU8 : nullptr, m.maxPx * 4, ncclUint8, 0, m.comms[r], m.streams[r]),
                       "ncclGather");
            nccl_check(ncclGather(m.sendF32[r], r == 0 ? m.recvF32 : nullptr, m.maxPx * 3, ncclFloat32, 0, m.comms[r],
                                  m.streams[r]), "ncclGather");
        }
        nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        for (int r = 0; r < world; ++r) {
            hip_check(hipSetDevice(devices[r]), "hipSetDevice");
            hip_check(hipStreamSynchronize(m.streams[r]), "hipStreamSynchronize");
        }
        hip_check(hipSetDevice(devices[0]), "hipSetDevice");
        hip_check(hipMemcpy(u8.data(), m.recvU8, u8.size(), hipMemcpyDeviceToHost), "hipMemcpy");
        hip_check(hipMemcpy(f32.data(), m.recvF32, f32.size() * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    } else {
        for (int r = 0; r < world; ++r) {
            hip_check(hipSetDevice(devices[r]), "hipSetDevice");
            hip_check(hipStreamSynchronize(m.streams[r]), "hipStreamSynchronize");
            hip_check(hipMemcpy(&u8[(size_t)r * m.maxPx * 4], m.sendU8[r], m.npx[r] * 4, hipMemcpyDeviceToHost), "hipMemcpy");
            hip_check(hipMemcpy(&f32[(size_t)r * m.maxPx * 3], m.sendF32[r], m.npx[r] * 12, hipMemcpyDeviceToHost), "hipMemcpy");
        }
    }
    for (int r = 0; r < world; ++r) check(m.ctx[r], pbr_hip_sync(m.ctx[r]), "pbr_hip_sync");   // deferred failures
    // scatter into the row-major frame, then into the FrameBuffer (flipped, Integrator.cpp:341-344)
    std::vector<uint8_t> frameU8((size_t)W * H * 4);
    std::vector<float> frameF((size_t)W * H * 3);
    for (int r = 0; r < world; ++r) {
        AssembleTiles(m.tiles[r], &u8[(size_t)r * m.maxPx * 4], 4, W, frameU8.data());
        AssembleTiles(m.tiles[r], &f32[(size_t)r * m.maxPx * 3], 3, W, frameF.data());
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int ch = 0; ch < m_FrameBuffer->channals; ++ch) {
                const size_t k = (size_t)y * W + x;
                m_FrameBuffer->set_uc(x, H - y - 1, ch, frameU8[4 * k + ch]);
                m_FrameBuffer->set_fc(x, H - y - 1, ch, ch < 3 ? frameF[3 * k + ch] : 1.f);
            }
    stats.samples = (uint64_t)W * H * (uint64_t)rd.spp;
    timeConsume = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    stats.seconds = timeConsume;
    stats.kernel_ms = 0;
    IntegratorRenderTime = (float)timeConsume;
}

}  // namespace PBR
