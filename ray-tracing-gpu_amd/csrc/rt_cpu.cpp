// rt_cpu.cpp — the CPU backend of the C ABI (include/rt.h, rt_create_cpu /
// rt_cpu_render*): SURVEY.md 8(b)'s second backend, the reference's CPU
// branch of CScene::LancerRayons (Scene.cpp:1535-1563) behind the same
// boundary, so a caller can switch backends the way the reference switched on
// CVar::g_ComputerShadersON (Var.cpp:11).  Explicit only: rt_create never
// returns a CPU context and the HIP entry points refuse one.
//
// Same images as the HIP kernel, bit for bit, by the same arguments:
//  * closest hit = the lexicographic minimum over (t, file index) of the
//    per-kind loops (the reference's strict '<' in file order, Scene.cpp:1713);
//  * shadow rays: when every filter factor (colour x Kt) is finite and >= +0,
//    meeting any opaque surface makes the filter exactly (+0, +0, +0) in any
//    multiplication order, so opaque surfaces are an any-hit test and the
//    translucent factors are multiplied in file order (Scene.cpp:1842-1861);
//    otherwise the generic file-order product;
//  * every expression in the reference's operand order (rt_math.h), IEEE
//    division and sqrt, no FMA contraction (the build's -ffp-contract=off).
// Work: 8-row bands of the output handed to host threads from an atomic
// counter.  Brute force over the surfaces (the reference's algorithm): the
// GPU path's culling structures are not rebuilt on the host.
#include "rt_cpu.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "rt_math.h"

#pragma clang fp contract(off)

namespace rt {
namespace cpu {

struct Tri {
    Vec3 p0, p1, p2, n;
    int file;
};
struct Plane {
    Vec3 n;
    float cst;
    int file;
};
struct Quad {
    Vec3 q, lin, mix;
    float cst;
    int file;
};
struct Material {
    Color color;
    float ka, kd, ks, shin, kr, kt, ior;
    Color filt;  // colour x Kt: the shadow filter factor (Scene.cpp:1855)
};
struct Light {
    Vec3 pos;
    Color color;
    float intens;
};

struct Scene {
    std::vector<int> kind, slot;  // file order: kind and index into its array
    std::vector<Tri> tri;
    std::vector<Plane> pla;
    std::vector<Quad> qua;
    std::vector<Material> mat;    // file order
    std::vector<Light> lights;
    std::vector<int> opaque, translucent;  // file indices
    bool split = false;
    float k_max = 0.0f;
};

struct Hit {
    float t = -1.0f;
    int file = -1;
};

// Triangle.cpp:127-172 (edges per test, as the reference computes them)
static bool hit_tri(const Tri& s, Vec3 O, Vec3 D, float& t)
{
    const Vec3 e1 = s.p1 - s.p0, e2 = s.p2 - s.p0;
    const Vec3 P = cross(D, e2);
    const float det = dot(e1, P);
    if (fabsf(det) < kEps) return false;
    const float inv = 1.0f / det;
    const Vec3 S = O - s.p0;
    const float u = dot(S, P) * inv;
    if (u < 0 || u > 1) return false;
    const Vec3 Q = cross(S, e1);
    const float v = dot(D, Q) * inv;
    if (v < 0 || u + v > 1) return false;
    t = dot(e2, Q) * inv;
    return true;
}

// Plan.cpp:128-144
static bool hit_plane(const Plane& s, Vec3 O, Vec3 D, float& t)
{
    const float vd = dot(s.n, D);
    if (!(fabsf(vd) > kEps)) return false;
    t = -(dot(s.n, O) + s.cst) / vd;
    return true;
}

// Quadrique.cpp:160-249: coefficient trees verbatim; min root, else the max
// if the min is below EPSILON, accepted if !(t < 0); A == 0: -0.5 (C / B).
static void quad_coef(const Quad& s, Vec3 o, Vec3 d, float& A, float& B, float& C)
{
    const Vec3 q = s.q, m = s.mix, l = s.lin;
    A = d.x * (q.x * d.x + m.z * d.y + m.y * d.z) + d.y * (q.y * d.y + m.x * d.z) + d.z * (q.z * d.z);
    B = d.x * (q.x * o.x + 0.5f * (m.z * o.y + m.y * o.z + l.x)) +
        d.y * (q.y * o.y + 0.5f * (m.z * o.x + m.x * o.z + l.y)) +
        d.z * (q.z * o.z + 0.5f * (m.y * o.x + m.x * o.y + l.z));
    C = o.x * (q.x * o.x + m.z * o.y + m.y * o.z + l.x) + o.y * (q.y * o.y + m.x * o.z + l.y) +
        o.z * (q.z * o.z + l.z) + s.cst;
}
static bool hit_quad(const Quad& s, Vec3 O, Vec3 D, float& t)
{
    float A, B, C;
    quad_coef(s, O, D, A, B, C);
    if (A != 0.0f) {
        const float Ka = -B / A, Kb = C / A;
        float delta = Ka * Ka - Kb;
        if (!(delta > 0)) return false;
        delta = sqrtf(delta);
        const float t0 = Ka - delta, t1 = Ka + delta;
        float dist = t0 < t1 ? t0 : t1;
        if (dist < kEps) dist = t0 > t1 ? t0 : t1;
        if (dist < 0) return false;
        t = dist;
        return true;
    }
    t = -0.5f * (C / B);
    return true;
}
static Vec3 quad_normal(const Quad& s, Vec3 O, Vec3 D, float t)
{
    float A, B, C;
    quad_coef(s, O, D, A, B, C);
    if (A != 0.0f) {
        const Vec3 hp = O + t * D;
        const Vec3 q = s.q, m = s.mix, l = s.lin;
        Vec3 n;
        n.x = 2.0f * q.x * hp.x + m.y * hp.z + m.z * hp.y + l.x;
        n.y = 2.0f * q.y * hp.y + m.x * hp.z + m.z * hp.x + l.y;
        n.z = 2.0f * q.z * hp.z + m.x * hp.y + m.y * hp.x + l.z;
        return normalize(n);
    }
    return normalize(s.lin);
}

static inline void take(bool ok, float t, int file, Hit& h)
{
    if (ok && t > kEps && (h.file < 0 || t < h.t || (t == h.t && file < h.file))) {
        h.t = t;
        h.file = file;
    }
}

// Scene.cpp:1705-1720 ObtenirCouleur's search
static Hit closest(const Scene& S, Vec3 O, Vec3 D)
{
    Hit h;
    float t = 0.0f;
    for (const Tri& s : S.tri) {
        const bool ok = hit_tri(s, O, D, t);
        take(ok, t, s.file, h);
    }
    for (const Plane& s : S.pla) {
        const bool ok = hit_plane(s, O, D, t);
        take(ok, t, s.file, h);
    }
    for (const Quad& s : S.qua) {
        const bool ok = hit_quad(s, O, D, t);
        take(ok, t, s.file, h);
    }
    return h;
}

static bool hit_file(const Scene& S, int i, Vec3 O, Vec3 D, float& t)
{
    const int k = S.slot[i];
    switch (S.kind[i]) {
    case RT_TRIANGLE: return hit_tri(S.tri[k], O, D, t);
    case RT_PLANE: return hit_plane(S.pla[k], O, D, t);
    default: return hit_quad(S.qua[k], O, D, t);
    }
}

static Vec3 normal_of(const Scene& S, int i, Vec3 O, Vec3 D, float t)
{
    const int k = S.slot[i];
    switch (S.kind[i]) {
    case RT_TRIANGLE: return S.tri[k].n;
    case RT_PLANE: return S.pla[k].n;
    default: return quad_normal(S.qua[k], O, D, t);
    }
}

// Scene.cpp:1842-1861 ObtenirFiltreDeSurface; L (unnormalised) is normalised
// in place like the reference's ray.
static Color filter(const Scene& S, Vec3 P, Vec3& L)
{
    const float dist = norm(L);
    L = div_recip(L, dist);
    Color F{1.0f, 1.0f, 1.0f};
    float t = 0.0f;
    if (!S.split) {
        for (size_t i = 0; i < S.kind.size(); ++i)
            if (hit_file(S, (int)i, P, L, t) && t > kEps && t < dist) F *= S.mat[i].filt;
        return F;
    }
    for (int i : S.opaque)
        if (hit_file(S, i, P, L, t) && t > kEps && t < dist) return Color{0.0f, 0.0f, 0.0f};
    for (int i : S.translucent)
        if (hit_file(S, i, P, L, t) && t > kEps && t < dist) F *= S.mat[i].filt;
    return F;
}

struct Ray {
    Vec3 O, D;
    float ior, energy;
    int bounces;
};

// Scene.cpp:1705-1826: colour of a ray, with the commented reflect / refract
// block (:1779-1823) re-enabled below max_bounces as the GPU path does.
static Color trace(const Scene& S, const rt_frame& f, const Ray& r)
{
    const Hit h = closest(S, r.O, r.D);
    if (h.file < 0) return Color{f.background[0], f.background[1], f.background[2]};
    const Material& m = S.mat[h.file];
    const Vec3 N = normal_of(S, h.file, r.O, r.D, h.t);
    const Vec3 P = r.O + h.t * r.D;
    Color res = m.color * m.ka;
    for (const Light& l : S.lights) {
        Vec3 L = l.pos - P;
        if (!(dot(L, N) > 0)) continue;  // Scene.cpp:1756, unnormalised
        const Color F = filter(S, P, L);
        const Color LC = l.color * F;
        const float g = l.intens * m.kd * dot(N, L);
        res += (m.color * g) * LC;
        const Vec3 rf = reflect(L, N);
        const float ps = dot(rf, r.D);
        if (ps > 0) {
            const float pf = l.intens * m.ks * powf(ps, m.shin);
            res += LC * pf;
        }
    }
    const float er = m.kr * r.energy, et = m.kt * r.energy;
    const bool can = r.bounces < f.max_bounces;
    if (er > f.min_energy && can) {  // reflected ray keeps CRayon's default IOR 0
        const Ray c{P, reflect(r.D, N), 0.0f, er, r.bounces + 1};
        res += trace(S, f, c) * m.kr;
    }
    if (et > f.min_energy && can) {
        Vec3 n = N;
        float ratio, ior;
        if (r.ior == m.ior) {  // inside -> out
            ior = f.scene_ior;
            ratio = m.ior / f.scene_ior;
            n = -n;
        } else {
            ior = m.ior;
            ratio = f.scene_ior / m.ior;
        }
        const Ray c{P, refract(r.D, n, ratio), ior, et, r.bounces + 1};
        res += trace(S, f, c) * m.kt;
    }
    return res;
}

// Scene.cpp:1543-1552 (the GPU's camera_dir, evaluated with IEEE sqrt and
// division: the same bits)
static Vec3 camera_dir(const rt_frame& f, int px, int py)
{
    const Vec3 d0 = make3((2 * px * f.inv_w - 1) * f.half_w, (2 * py * f.inv_h - 1) * f.half_h, -1.0f);
    Mat4 M;
    for (int i = 0; i < 16; ++i) M.m[i >> 2][i & 3] = f.orient[i];
    return normalize(d0 * M);
}

}  // namespace cpu

int cpu_upload(void** handle, const rt_scene_flat* s)
{
    using namespace cpu;
    Scene* S = new Scene();
    const int n = s->n_surfaces;
    bool split = true;
    for (int i = 0; i < n; ++i) {
        const float* g = s->geom + 12 * (size_t)i;
        const float* m = s->material + 10 * (size_t)i;
        const int kind = s->type[i];
        if (kind < RT_TRIANGLE || kind > RT_QUADRIC) {
            delete S;
            return RT_E_ARG;
        }
        S->kind.push_back(kind);
        if (kind == RT_TRIANGLE) {
            S->slot.push_back((int)S->tri.size());
            S->tri.push_back(Tri{make3(g[0], g[1], g[2]), make3(g[3], g[4], g[5]), make3(g[6], g[7], g[8]),
                                 make3(g[9], g[10], g[11]), i});
        } else if (kind == RT_PLANE) {
            S->slot.push_back((int)S->pla.size());
            S->pla.push_back(Plane{make3(g[0], g[1], g[2]), g[3], i});
        } else {
            S->slot.push_back((int)S->qua.size());
            S->qua.push_back(Quad{make3(g[0], g[1], g[2]), make3(g[3], g[4], g[5]), make3(g[6], g[7], g[8]), g[9], i});
        }
        Material q{Color{m[0], m[1], m[2]}, m[3], m[4], m[5], m[6], m[7], m[8], m[9], Color{0, 0, 0}};
        q.filt = q.color * q.kt;
        auto ok = [](float v) { return std::isfinite(v) && !std::signbit(v); };
        split = split && ok(q.filt.r) && ok(q.filt.g) && ok(q.filt.b);
        S->mat.push_back(q);
        if (q.filt.r == 0.0f && q.filt.g == 0.0f && q.filt.b == 0.0f)
            S->opaque.push_back(i);
        else
            S->translucent.push_back(i);
    }
    for (int j = 0; j < s->n_lights; ++j) {
        const float* l = s->lights + 7 * (size_t)j;
        S->lights.push_back(Light{make3(l[0], l[1], l[2]), Color{l[3], l[4], l[5]}, l[6]});
    }
    S->split = split;
    cpu_free(*handle);
    *handle = S;
    return RT_OK;
}

void cpu_free(void* handle) { delete static_cast<cpu::Scene*>(handle); }

// Output row q of frame f -> frame row (the slab, or the band set).
static int out_row(const rt_frame& f, int q)
{
    if (f.band_rows == 0) return f.row_begin + q;
    const int b = q / f.band_rows;
    return (b * f.band_count + f.band_index) * f.band_rows + q % f.band_rows;
}

int cpu_render(const void* handle, int threads, const rt_frame* f, int rows, uint8_t* rgba, float* rgb, double* ms)
{
    using namespace cpu;
    const Scene& S = *static_cast<const Scene*>(handle);
    const auto t0 = std::chrono::steady_clock::now();
    const int W = f->width;
    std::atomic<int> next{0};
    constexpr int kBand = 8;
    auto work = [&]() {
        for (;;) {
            const int q0 = next.fetch_add(kBand);
            if (q0 >= rows) return;
            for (int q = q0; q < std::min(rows, q0 + kBand); ++q) {
                const int y = out_row(*f, q);
                for (int x = 0; x < W; ++x) {
                    const size_t o = (size_t)q * W + x;
                    if (y >= f->height) {  // a band row past the frame: left unwritten, like the kernel
                        continue;
                    }
                    const Ray r{make3(f->cam_pos[0], f->cam_pos[1], f->cam_pos[2]), camera_dir(*f, x, y), 1.0f,
                                1.0f, 0};
                    const Color c = trace(S, *f, r);
                    if (rgb) {
                        rgb[3 * o] = c.r;
                        rgb[3 * o + 1] = c.g;
                        rgb[3 * o + 2] = c.b;
                    }
                    if (rgba) {
                        rgba[4 * o] = (uint8_t)unorm8(c.r);
                        rgba[4 * o + 1] = (uint8_t)unorm8(c.g);
                        rgba[4 * o + 2] = (uint8_t)unorm8(c.b);
                        rgba[4 * o + 3] = 255;
                    }
                }
            }
        }
    };
    int n = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    n = std::max(1, std::min(n, (rows + kBand - 1) / kBand));
    std::vector<std::thread> pool;
    for (int i = 1; i < n; ++i) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

}  // namespace rt
