// rt_bvhhost.h — host build of the bounce-ray BVH (rt_bvh.h), at upload.
// Part of the host half of rt_kernels.hip (included after rt_ctx).
//
// A binned-SAH BVH2 over every triangle of tri[] (opaque and translucent:
// closest hit does not care), leaves of at most 4 triangles, inner nodes
// in depth-first order.  Each child box is the union of its triangles' boxes
// — the float vertices p0, p0 + e1, p0 + e2 the reference's test uses,
// summed in double and rounded outwards to float — with the largest alpha
// of its triangles (rt_bvh.h's margin bound), rounded up.
#ifndef RT_AMD_RT_BVHHOST_H
#define RT_AMD_RT_BVHHOST_H

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace rt {

constexpr int kBvhLeafMax = 4;
constexpr int kBvhMedianDepth = 20;  // past this depth: median splits

// Levels of median splits below a node of m triangles: ceil(log2(ceil(m / 4))).
inline int bvh_median_levels(size_t m)
{
    int k = 0;
    for (size_t cap = kBvhLeafMax; cap < m; cap *= 2) ++k;
    return k;
}

struct BvhPrim {
    float lo[3], hi[3];
    double c[3];    // centroid (binning)
    float alpha;    // eps (40 K + 36), raised for the box test's rounding; +inf: never culled
};

struct BvhBuilt {
    std::vector<float4> nodes;  // 4 per inner node
    std::vector<float4> tris;   // 3 per triangle, leaf order
    int depth = 0, leaves = 0, inner = 0;
};

// rt_bvh.h's per-triangle margin coefficients, in double, rounded up.
inline void bvh_prim(const float* r, BvhPrim& p)
{
    const double eps = 0x1p-24;
    double v[3][3];
    for (int a = 0; a < 3; ++a) {
        v[0][a] = r[a];
        v[1][a] = (double)r[a] + (double)r[3 + a];
        v[2][a] = (double)r[a] + (double)r[6 + a];
    }
    for (int a = 0; a < 3; ++a) {
        const double lo = std::min(v[0][a], std::min(v[1][a], v[2][a]));
        const double hi = std::max(v[0][a], std::max(v[1][a], v[2][a]));
        p.lo[a] = std::nextafter((float)lo, -INFINITY);
        p.hi[a] = std::nextafter((float)hi, INFINITY);
        p.c[a] = 0.5 * (lo + hi);
        if (!std::isfinite(p.c[a])) p.c[a] = 0.0;
    }
    const double n1 = std::sqrt((double)r[3] * r[3] + (double)r[4] * r[4] + (double)r[5] * r[5]);
    const double n2 = std::sqrt((double)r[6] * r[6] + (double)r[7] * r[7] + (double)r[8] * r[8]);
    const double prod = n1 * n2 * (1.0 + 1e-12);
    const double den = 0.01 - 6.1 * eps * 1.01 * prod;
    double alpha = INFINITY;
    if (den > 0.001 && std::isfinite(prod)) {
        const double K = 1.01 * prod / den;
        alpha = eps * (40.0 * K + 4.0 + 32.0) * (1.0 + 1e-5) + 1e-6;  // + 32 eps: the 16 eps L term
    }
    const bool finite_box = std::isfinite(p.lo[0]) && std::isfinite(p.lo[1]) && std::isfinite(p.lo[2]) &&
                            std::isfinite(p.hi[0]) && std::isfinite(p.hi[1]) && std::isfinite(p.hi[2]);
    if (!finite_box || !(alpha < 1.0)) alpha = INFINITY;
    p.alpha = std::isfinite(alpha) ? std::nextafter((float)alpha, INFINITY) : INFINITY;
}

struct BvhBox {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float alpha = 0.f;
    void add(const BvhPrim& p)
    {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p.lo[a]);
            hi[a] = std::max(hi[a], p.hi[a]);
        }
        alpha = std::max(alpha, p.alpha);
    }
    double area() const
    {
        const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        return dx * dy + dy * dz + dz * dx;
    }
};

class BvhBuilder {
  public:
    BvhBuilder(const std::vector<BvhPrim>& prims, std::vector<int>& ord) : P(prims), ord(ord) {}
    // builds [b, e) (more than kBvhLeafMax triangles) as inner node `at`
    void inner(int at, size_t b, size_t e, int depth, BvhBuilt& out)
    {
        out.depth = std::max(out.depth, depth + 1);
        const size_t mid = split(b, e, depth);
        float4* n = &out.nodes[4 * (size_t)at];
        int refs[2];
        const size_t rb[2] = {b, mid}, re[2] = {mid, e};
        for (int c = 0; c < 2; ++c) {
            BvhBox bx;
            for (size_t i = rb[c]; i < re[c]; ++i) bx.add(P[ord[i]]);
            n = &out.nodes[4 * (size_t)at];  // (the vector may have grown)
            n[2 * c] = make_float4(bx.lo[0], bx.lo[1], bx.lo[2], bx.alpha);
            n[2 * c + 1] = make_float4(bx.hi[0], bx.hi[1], bx.hi[2], 0.f);
            const size_t cnt = re[c] - rb[c];
            if (cnt <= (size_t)kBvhLeafMax) {
                refs[c] = (int)~(((unsigned)rb[c] << 4) | (unsigned)(cnt - 1));
                ++out.leaves;
                out.depth = std::max(out.depth, depth + 1);
            } else {
                const int child = (int)(out.nodes.size() / 4);
                out.nodes.resize(out.nodes.size() + 4, make_float4(0.f, 0.f, 0.f, 0.f));
                refs[c] = child;
                inner(child, rb[c], re[c], depth + 1, out);
            }
            n = &out.nodes[4 * (size_t)at];
            std::memcpy(&n[2 * c + 1].w, &refs[c], sizeof(int));
        }
        ++out.inner;
    }

  private:
    const std::vector<BvhPrim>& P;
    std::vector<int>& ord;

    // Binned SAH (16 bins on the widest centroid axis); median split past
    // kBvhMedianDepth or when every centroid coincides.
    size_t split(size_t b, size_t e, int depth)
    {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], P[ord[i]].c[a]);
                hi[a] = std::max(hi[a], P[ord[i]].c[a]);
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a)
            if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        const size_t half = b + (e - b) / 2;
        auto median = [&]() {
            std::nth_element(ord.begin() + b, ord.begin() + half, ord.begin() + e, [&](int x, int y) {
                return P[x].c[ax] < P[y].c[ax] || (P[x].c[ax] == P[y].c[ax] && x < y);
            });
            return half;
        };
        const double ext = hi[ax] - lo[ax];
        if (depth >= kBvhMedianDepth || !(ext > 0.0)) return median();
        constexpr int NB = 16;
        BvhBox bins[NB];
        size_t cnt[NB] = {};
        auto bin_of = [&](int k) {
            const int q = (int)((P[k].c[ax] - lo[ax]) / ext * NB);
            return std::min(NB - 1, std::max(0, q));
        };
        for (size_t i = b; i < e; ++i) {
            const int q = bin_of(ord[i]);
            bins[q].add(P[ord[i]]);
            ++cnt[q];
        }
        double left_area[NB], best = INFINITY;
        size_t left_cnt[NB];
        BvhBox acc;
        size_t na = 0;
        for (int q = 0; q < NB; ++q) {
            if (cnt[q]) {
                for (int a = 0; a < 3; ++a) {
                    acc.lo[a] = std::min(acc.lo[a], bins[q].lo[a]);
                    acc.hi[a] = std::max(acc.hi[a], bins[q].hi[a]);
                }
            }
            na += cnt[q];
            left_area[q] = acc.area();
            left_cnt[q] = na;
        }
        BvhBox racc;
        size_t nr = 0;
        int cut = -1;
        for (int q = NB - 1; q > 0; --q) {  // split between bin q-1 and q
            if (cnt[q]) {
                for (int a = 0; a < 3; ++a) {
                    racc.lo[a] = std::min(racc.lo[a], bins[q].lo[a]);
                    racc.hi[a] = std::max(racc.hi[a], bins[q].hi[a]);
                }
            }
            nr += cnt[q];
            const size_t nl = left_cnt[q - 1];
            if (nl == 0 || nr == 0) continue;
            const double cost = left_area[q - 1] * (double)nl + racc.area() * (double)nr;
            if (cost < best) {
                best = cost;
                cut = q;
            }
        }
        if (cut < 0) return median();
        const auto it = std::partition(ord.begin() + b, ord.begin() + e, [&](int k) { return bin_of(k) < cut; });
        const size_t mid = (size_t)(it - ord.begin());
        if (mid == b || mid == e) return median();
        // Depth bound: every node keeps depth + bvh_median_levels(count) <=
        // kBvhStack (the root does for up to 4 x 2^24 triangles); an SAH cut
        // whose larger side would break it is replaced by the median cut,
        // which keeps it — so the tree always fits the walk's stack.
        if (depth + 1 + bvh_median_levels(std::max(mid - b, e - mid)) > kBvhStack) return median();
        return mid;
    }
};

// Largest triangle count the leaf encoding ~((first << 4) | (count - 1))
// keeps negative (first < 2^27) and the median-split bound keeps within
// kBvhStack levels (4 x 2^24): larger scenes trace bounce rays without a BVH.
constexpr size_t kBvhMaxTriangles = (size_t)kBvhLeafMax << kBvhStack;
static_assert(kBvhMaxTriangles <= ((size_t)1 << 27), "leaf encoding");

// The BVH over tri[] (12 floats per triangle, kBvhLeafMax < n <= kBvhMaxTriangles).
inline void bvh_build(const std::vector<float>& tri, size_t n, BvhBuilt& out)
{
    std::vector<BvhPrim> P(n);
    for (size_t k = 0; k < n; ++k) bvh_prim(&tri[12 * k], P[k]);
    std::vector<int> ord(n);
    for (size_t k = 0; k < n; ++k) ord[k] = (int)k;
    out = BvhBuilt{};
    out.nodes.resize(4, make_float4(0.f, 0.f, 0.f, 0.f));
    BvhBuilder(P, ord).inner(0, 0, n, 0, out);
    out.tris.resize(3 * n);
    for (size_t i = 0; i < n; ++i) std::memcpy(&out.tris[3 * i], &tri[12 * (size_t)ord[i]], 12 * sizeof(float));
}

}  // namespace rt
#endif  // RT_AMD_RT_BVHHOST_H
