// pbr_xform.h — row-major 4x4 transform math shared by the device library's scene/camera setup
// (pbr_scene.cpp) and the C++ host API (host/), so both produce the same bits
// (Core/Transform.cpp: Matrix4x4::Inverse, operator*, Scale, Translate, Perspective, LookAt).
#pragma once
#include <cmath>
#include <cstring>
#include <utility>

#include "pbr_math.h"

namespace pbr {
namespace xform {

// Row-major 4x4 helpers for the camera/transform math (Core/Transform.*).
struct Mat { float a[4][4]; };
inline Mat identity() { Mat m; for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) m.a[i][j] = i == j ? 1.f : 0.f; return m; }
inline Mat from_rows(const float* r) { Mat m; std::memcpy(m.a, r, 64); return m; }
inline Mat mul(const Mat& x, const Mat& y) {
    Mat r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.a[i][j] = x.a[i][0] * y.a[0][j] + x.a[i][1] * y.a[1][j] + x.a[i][2] * y.a[2][j] + x.a[i][3] * y.a[3][j];
    return r;
}
// Gauss-Jordan elimination with full pivoting, float arithmetic (Transform.cpp:59-130)
inline Mat invert(const Mat& in) {
    int colOf[4], rowOf[4], used[4] = {0, 0, 0, 0};
    float w[4][4];
    std::memcpy(w, in.a, 64);
    for (int step = 0; step < 4; ++step) {
        int prow = 0, pcol = 0;
        float best = 0.f;
        for (int r = 0; r < 4; ++r) {
            if (used[r] == 1) continue;
            for (int c = 0; c < 4; ++c)
                if (used[c] == 0 && std::fabs(w[r][c]) >= best) { best = std::fabs(w[r][c]); prow = r; pcol = c; }
        }
        ++used[pcol];
        if (prow != pcol) for (int c = 0; c < 4; ++c) std::swap(w[prow][c], w[pcol][c]);
        rowOf[step] = prow;
        colOf[step] = pcol;
        float inv = 1. / w[pcol][pcol];
        w[pcol][pcol] = 1.;
        for (int c = 0; c < 4; ++c) w[pcol][c] *= inv;
        for (int r = 0; r < 4; ++r) {
            if (r == pcol) continue;
            float f = w[r][pcol];
            w[r][pcol] = 0;
            for (int c = 0; c < 4; ++c) w[r][c] -= w[pcol][c] * f;
        }
    }
    for (int k = 3; k >= 0; --k)
        if (rowOf[k] != colOf[k])
            for (int r = 0; r < 4; ++r) std::swap(w[r][rowOf[k]], w[r][colOf[k]]);
    Mat m;
    std::memcpy(m.a, w, 64);
    return m;
}
struct Xf { Mat m, mi; };
inline Xf compose(const Xf& x, const Xf& y) { return Xf{mul(x.m, y.m), mul(y.mi, x.mi)}; }   // Transform::operator*
inline Xf inverse(const Xf& x) { return Xf{x.mi, x.m}; }
inline Xf scale(float x, float y, float z) {
    Xf t{identity(), identity()};
    t.m.a[0][0] = x; t.m.a[1][1] = y; t.m.a[2][2] = z;
    t.mi.a[0][0] = 1 / x; t.mi.a[1][1] = 1 / y; t.mi.a[2][2] = 1 / z;
    return t;
}
inline Xf translate(f3 d) {
    Xf t{identity(), identity()};
    t.m.a[0][3] = d.x; t.m.a[1][3] = d.y; t.m.a[2][3] = d.z;
    t.mi.a[0][3] = -d.x; t.mi.a[1][3] = -d.y; t.mi.a[2][3] = -d.z;
    return t;
}
inline Xf perspective(float fovDeg, float n, float f) {   // Transform.cpp:257-264
    Mat p = identity();
    p.a[2][2] = f / (f - n);
    p.a[2][3] = -f * n / (f - n);
    p.a[3][2] = 1;
    p.a[3][3] = 0;
    float half = ((kPi / 180) * fovDeg) / 2;
    float invTanAng = 1 / (float)tan((double)half);
    return compose(scale(invTanAng, invTanAng, 1), Xf{p, invert(p)});
}
inline Xf look_at(f3 pos, f3 look, f3 up) {   // Transform.cpp:208-239 (world → camera)
    Mat c = identity();
    c.a[0][3] = pos.x; c.a[1][3] = pos.y; c.a[2][3] = pos.z; c.a[3][3] = 1;
    f3 dir = normalize(look - pos);
    if (len(cross(normalize(up), dir)) == 0) return Xf{identity(), identity()};
    f3 right = normalize(cross(normalize(up), dir));
    f3 newUp = cross(dir, right);
    c.a[0][0] = right.x; c.a[1][0] = right.y; c.a[2][0] = right.z; c.a[3][0] = 0.;
    c.a[0][1] = newUp.x; c.a[1][1] = newUp.y; c.a[2][1] = newUp.z; c.a[3][1] = 0.;
    c.a[0][2] = dir.x; c.a[1][2] = dir.y; c.a[2][2] = dir.z; c.a[3][2] = 0.;
    return Xf{invert(c), c};
}
inline bool swaps_handedness(const Mat& m) {   // Transform.cpp:144-150
    float det = m.a[0][0] * (m.a[1][1] * m.a[2][2] - m.a[1][2] * m.a[2][1]) -
                m.a[0][1] * (m.a[1][0] * m.a[2][2] - m.a[1][2] * m.a[2][0]) +
                m.a[0][2] * (m.a[1][0] * m.a[2][1] - m.a[1][1] * m.a[2][0]);
    return det < 0;
}


}  // namespace xform
}  // namespace pbr
