// rt_math.h — Math3D for the MI355X ray tracer, usable on host and device.
//
// A re-implementation of the reference's Math3D layer (MathUtils.h,
// Vecteur3.h, Matrice4.h/.cpp, Couleur.h) whose only contract is the
// reference's floating-point EVALUATION ORDER:
// REAL = float (MathUtils.h:23), left-to-right sums, no FMA contraction,
// IEEE division except where the reference multiplies by a reciprocal.
// The parity of every expression below is pinned by tests/ against the
// oracle and the golden fixtures produced from the reference's own sources.
#pragma once

#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

#pragma clang fp contract(off)

namespace rt {

constexpr float kEps = 1.0e-2f;            // MathUtils.h:35 EPSILON
constexpr float kPi = (float)3.14159265358979323846; // (float)M_PI, MathUtils.h:28-32
constexpr float kInv255 = 1.0f / 255.0f;   // Couleur.cpp UBYTE_2_FLOAT

struct Vec3 {
    float x, y, z;
};

RT_HD Vec3 make3(float x, float y, float z) { return Vec3{x, y, z}; }
RT_HD Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD Vec3 operator-(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD Vec3 operator-(Vec3 a) { return {-a.x, -a.y, -a.z}; }
// Vecteur3.h operator*(REAL, V) == operator*(V, REAL): component * scalar
RT_HD Vec3 operator*(Vec3 v, float s) { return {v.x * s, v.y * s, v.z * s}; }
RT_HD Vec3 operator*(float s, Vec3 v) { return {v.x * s, v.y * s, v.z * s}; }
// Vecteur3.h ProdScal
RT_HD float dot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// Vecteur3.h ProdVect
RT_HD Vec3 cross(Vec3 a, Vec3 b)
{
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
RT_HD float norm(Vec3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
// Vecteur3.h operator/(REAL): one reciprocal, three multiplies
RT_HD Vec3 div_recip(Vec3 v, float s)
{
    const float inv = 1.0f / s;
    return {v.x * inv, v.y * inv, v.z * inv};
}
// Vecteur3.h Normaliser: zero vector when |v| <= EPSILON
RT_HD Vec3 normalize(Vec3 v)
{
    const float len = norm(v);
    if (len > kEps) {
        const float inv = 1.0f / len;
        return v * inv;
    }
    return {0.f, 0.f, 0.f};
}
// Vecteur3.h Reflect: v - (2*dot(v,n)) * n
RT_HD Vec3 reflect(Vec3 v, Vec3 n) { return v - (2.0f * dot(v, n)) * n; }
// Vecteur3.h Refract.  pow(float, int) promotes to double in C++11, so the
// cosine term is evaluated in double and narrowed once when it meets REAL.
RT_HD Vec3 refract(Vec3 v, Vec3 n, float eta)
{
    const Vec3 z = eta * (v - dot(v, n) * n);
    const double zn = (double)norm(z);
    const float c = (float)sqrt(1.0 - zn * zn);
    const Vec3 t = z - c * n;
    if (dot(t, n) < 0) return t;
    return reflect(v, n);
}

// Matrice4.h: row-major m[4][4], row-vector convention (v * M).
struct Mat4 {
    float m[4][4];
};
RT_HD Mat4 identity4()
{
    Mat4 r{};
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.0f;
    return r;
}
// Matrice4.h Concatene
RT_HD Mat4 operator*(const Mat4& a, const Mat4& b)
{
    Mat4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j] +
                        a.m[i][3] * b.m[3][j];
    return r;
}
// Matrice4.h operator*(CVecteur3, CMatrice4): affine point transform
RT_HD Vec3 operator*(Vec3 v, const Mat4& M)
{
    return {M.m[0][0] * v.x + M.m[1][0] * v.y + M.m[2][0] * v.z + M.m[3][0],
            M.m[0][1] * v.x + M.m[1][1] * v.y + M.m[2][1] * v.z + M.m[3][1],
            M.m[0][2] * v.x + M.m[1][2] * v.y + M.m[2][2] * v.z + M.m[3][2]};
}
RT_HD Mat4 transpose(const Mat4& a)
{
    Mat4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) r.m[i][j] = a.m[j][i];
    return r;
}
// Matrice4.cpp:29-106 — 2x2 sub-determinant expansion with the same
// temporaries in the same order.
RT_HD Mat4 inverse(const Mat4& M)
{
    const float a00 = M.m[0][0], a01 = M.m[0][1], a02 = M.m[0][2], a03 = M.m[0][3];
    const float a10 = M.m[1][0], a11 = M.m[1][1], a12 = M.m[1][2], a13 = M.m[1][3];
    const float a20 = M.m[2][0], a21 = M.m[2][1], a22 = M.m[2][2], a23 = M.m[2][3];
    const float a30 = M.m[3][0], a31 = M.m[3][1], a32 = M.m[3][2], a33 = M.m[3][3];
    Mat4 r;
    float s0 = a20 * a31 - a21 * a30, s1 = a20 * a32 - a22 * a30, s2 = a20 * a33 - a23 * a30;
    float s3 = a21 * a32 - a22 * a31, s4 = a21 * a33 - a23 * a31, s5 = a22 * a33 - a23 * a32;
    const float c00 = (s5 * a11 - s4 * a12 + s3 * a13);
    const float c10 = -(s5 * a10 - s2 * a12 + s1 * a13);
    const float c20 = (s4 * a10 - s2 * a11 + s0 * a13);
    const float c30 = -(s3 * a10 - s1 * a11 + s0 * a12);
    const float id = 1.0f / (c00 * a00 + c10 * a01 + c20 * a02 + c30 * a03);
    r.m[0][0] = c00 * id;
    r.m[1][0] = c10 * id;
    r.m[2][0] = c20 * id;
    r.m[3][0] = c30 * id;
    r.m[0][1] = -(s5 * a01 - s4 * a02 + s3 * a03) * id;
    r.m[1][1] = (s5 * a00 - s2 * a02 + s1 * a03) * id;
    r.m[2][1] = -(s4 * a00 - s2 * a01 + s0 * a03) * id;
    r.m[3][1] = (s3 * a00 - s1 * a01 + s0 * a02) * id;
    s0 = a10 * a31 - a11 * a30; s1 = a10 * a32 - a12 * a30; s2 = a10 * a33 - a13 * a30;
    s3 = a11 * a32 - a12 * a31; s4 = a11 * a33 - a13 * a31; s5 = a12 * a33 - a13 * a32;
    r.m[0][2] = (s5 * a01 - s4 * a02 + s3 * a03) * id;
    r.m[1][2] = -(s5 * a00 - s2 * a02 + s1 * a03) * id;
    r.m[2][2] = (s4 * a00 - s2 * a01 + s0 * a03) * id;
    r.m[3][2] = -(s3 * a00 - s1 * a01 + s0 * a02) * id;
    s0 = a21 * a10 - a20 * a11; s1 = a22 * a10 - a20 * a12; s2 = a23 * a10 - a20 * a13;
    s3 = a22 * a11 - a21 * a12; s4 = a23 * a11 - a21 * a13; s5 = a23 * a12 - a22 * a13;
    r.m[0][3] = -(s5 * a01 - s4 * a02 + s3 * a03) * id;
    r.m[1][3] = (s5 * a00 - s2 * a02 + s1 * a03) * id;
    r.m[2][3] = -(s4 * a00 - s2 * a01 + s0 * a03) * id;
    r.m[3][3] = (s3 * a00 - s1 * a01 + s0 * a02) * id;
    return r;
}

// Couleur.h — the colour algebra the shading uses.  Only operator+ clamps,
// and the shading path never calls it; += / *= / * never clamp.
struct Color {
    float r, g, b;
};
RT_HD Color rgb_from_int(int R, int G, int B) { return {R * kInv255, G * kInv255, B * kInv255}; }
RT_HD Color operator*(Color c, float s) { return {c.r * s, c.g * s, c.b * s}; }
RT_HD Color operator*(Color a, Color b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
RT_HD Color& operator+=(Color& a, Color b)
{
    a.r += b.r;
    a.g += b.g;
    a.b += b.b;
    return a;
}
RT_HD Color& operator*=(Color& a, Color b)
{
    a.r *= b.r;
    a.g *= b.g;
    a.b *= b.b;
    return a;
}

// MathUtils.h:132-136
RT_HD float deg2rad(float a) { return (a / 180.0f) * kPi; }

// GL's float -> GL_RGBA8 conversion for glTexImage2D(..., GL_FLOAT, ...)
// (Scene.cpp:1562): clamp to [0,1], scale by 255, round to nearest.  NaN -> 0.
RT_HD unsigned int unorm8(float f)
{
    const float c = f > 0.0f ? (f < 1.0f ? f : 1.0f) : 0.0f;
    return (unsigned int)floorf(c * 255.0f + 0.5f);
}

}  // namespace rt
