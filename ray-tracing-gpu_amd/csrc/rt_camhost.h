// rt_camhost.h — host half of the per-camera state: the camera buffer's
// build orchestration (rt_cambuf.h kernels: capacities from earlier builds,
// no host round trip) and the launch-camera path of tiny scenes (rt_cull.h
// TinyCam: records computed on the host, tile masks per stream).
// Part of the host code of rt_kernels.hip (one translation unit, included
// after struct rt_ctx and the stream-ordering helpers it uses).
#ifndef RT_AMD_RT_CAMHOST_H
#define RT_AMD_RT_CAMHOST_H

// ---- the camera buffer (rt_cambuf.h), host side
// A replaced buffer that an enqueued render or build may still read: freed
// at the next host sync of the context (or kept for a captured graph).
static void free_later(rt_ctx* c, void* p)
{
    if (!p) return;
    if (c->captured)
        c->retired.push_back(p);
    else
        c->deferred.push_back(p);
}

static void cb_free(rt_ctx::CamBuf& B)
{
    hipFree(B.tcone);
    hipFree(B.off);
    hipFree(B.cur);
    hipFree(B.flag);
    hipFree(B.box);
    hipFree(B.tcnt);
    hipFree(B.rmask);
    hipFree(B.lng);
    hipFree(B.mid);
    hipFree(B.stat);
    hipFree(B.scan);
    hipFree(B.ent);
    hipFree(B.rec);
    if (B.ev_tot) hipEventDestroy(B.ev_tot);
    if (B.ev0) hipEventDestroy(B.ev0);
    if (B.ev1) hipEventDestroy(B.ev1);
    B = rt_ctx::CamBuf{};
}

// The camera buffer needs the frame's orientation to be a rotation (rows
// 0-2 orthonormal to 1e-5, no translation row: cb_box reads directions in
// camera coordinates through it) and a sane film; other frames render
// without one (the per-wave path: the same image).
static bool cb_frame_ok(const rt_frame* f)
{
    const float* m = f->orient;
    if (m[12] != 0.0f || m[13] != 0.0f || m[14] != 0.0f) return false;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const double d = (double)m[4 * i] * m[4 * j] + (double)m[4 * i + 1] * m[4 * j + 1] +
                             (double)m[4 * i + 2] * m[4 * j + 2];
            if (!(std::fabs(d - (i == j ? 1.0 : 0.0)) <= 1e-5)) return false;
        }
    const float v[4] = {f->half_w, f->half_h, f->inv_w, f->inv_h};
    for (float x : v)
        if (!(x > 0.0f) || !std::isfinite(x)) return false;
    return true;
}

// Read back the last build's total and counters if its copy has landed
// (no wait).
static void cb_harvest(rt_ctx::CamBuf& B)
{
    if (!B.tot_pending || hipEventQuery(B.ev_tot) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    B.tot_pending = false;
    B.entries = (size_t)B.h_tot[0];
    B.observed = std::max(B.observed, B.entries);
    std::memcpy(B.hstat, B.h_tot + 1, sizeof B.hstat);
    if (!B.hstat[6]) B.observed_pairs = std::max(B.observed_pairs, (size_t)B.hstat[1]);
    // a build that did not fit (tiles sent down the per-wave path) is
    // rebuilt at its camera's next render, now that the sizes are known
    // (a build past 2^32 - 1 candidate pairs stays valid: every tile flagged)
    if (B.entries > B.built_cap || (!B.hstat[6] && ((size_t)B.hstat[1] + 63) / 64 > B.built_rcap)) B.valid = false;
}

// Per-tile arrays for nt tiles, the per-build words, the deferred-triangle
// list for the scene's triangles.
static int cb_ensure(rt_ctx* c, rt_ctx::CamBuf& B, int nt, bool capturing)
{
    if (!B.ev_tot) {
        HIP_TRY(c, hipEventCreateWithFlags(&B.ev_tot, hipEventDisableTiming));
        HIP_TRY(c, hipEventCreate(&B.ev0));
        HIP_TRY(c, hipEventCreate(&B.ev1));
        B.h_tot = c->h_cbwords + 8 * (c->n_cbwords++ % kCbWordSets);  // pinned words from rt_create
        HIP_TRY(c, hipMalloc((void**)&B.stat, 8 * sizeof(unsigned)));
    }
    if (nt > B.nt_alloc || c->n_tri > B.big_alloc) {
        free_later(c, B.tcone);
        free_later(c, B.off);
        free_later(c, B.cur);
        free_later(c, B.flag);
        free_later(c, B.lng);
        free_later(c, B.mid);
        free_later(c, B.scan);
        B.tcone = nullptr;
        B.off = B.cur = B.flag = nullptr;
        B.lng = B.mid = nullptr;
        B.scan = nullptr;
        B.nt_alloc = 0;
        HIP_TRY(c, hipMalloc((void**)&B.tcone, (size_t)nt * 2 * sizeof(float4)));
        HIP_TRY(c, hipMalloc((void**)&B.off, (size_t)(nt + 1) * sizeof(unsigned)));
        HIP_TRY(c, hipMalloc((void**)&B.cur, (size_t)nt * sizeof(unsigned)));
        HIP_TRY(c, hipMalloc((void**)&B.flag, (size_t)nt * sizeof(unsigned)));
        HIP_TRY(c, hipMalloc((void**)&B.lng, (size_t)nt * sizeof(int)));
        HIP_TRY(c, hipMalloc((void**)&B.mid, (size_t)nt * sizeof(int)));
        B.scan_words = scan_scratch((size_t)std::max(nt, c->n_tri));
        HIP_TRY(c, hipMalloc(&B.scan, B.scan_words * sizeof(unsigned long long)));
        B.nt_alloc = nt;
    }
    if (c->n_tri > B.big_alloc) {
        free_later(c, B.box);
        free_later(c, B.tcnt);
        B.box = nullptr;
        B.tcnt = nullptr;
        B.big_alloc = 0;
        HIP_TRY(c, hipMalloc((void**)&B.box, (size_t)c->n_tri * sizeof(int4)));
        HIP_TRY(c, hipMalloc((void**)&B.tcnt, (size_t)(c->n_tri + 1) * sizeof(unsigned)));
        B.big_alloc = c->n_tri;
    }
    // pass masks: 1.25 x the largest candidate count read back, or a first
    // guess of 64 candidates per triangle
    const size_t runs = B.observed_pairs ? (B.observed_pairs / 64) * 5 / 4 + 1024
                                         : std::max<size_t>(16384, (size_t)c->n_tri);
    if (runs > B.rcap && !capturing) {  // a capture keeps the masks it has (the runs past them: per-wave)
        free_later(c, B.rmask);
        B.rmask = nullptr;
        B.rcap = 0;
        HIP_TRY(c, hipMalloc((void**)&B.rmask, runs * sizeof(unsigned long long)));
        B.rcap = runs;
    }
    return RT_OK;
}

static int cb_grow(rt_ctx* c, rt_ctx::CamBuf& B, size_t want)
{
    if (want <= B.cap && B.ent) return RT_OK;
    if (want > 0xFFFFFFF0ull) {
        c->err = "camera buffer too large";
        return RT_E_UNSUPPORTED;
    }
    free_later(c, B.ent);
    B.ent = nullptr;
    B.cap = 0;
    HIP_TRY(c, hipMalloc((void**)&B.ent, std::max<size_t>(want, 1) * sizeof(int2)));
    B.cap = std::max<size_t>(want, 1);
    return RT_OK;
}

// Entries a build should have room for: 1.25 x the largest total read back
// (plus slack), or a first guess of 16 per tile.
static size_t cb_want_cap(const rt_ctx::CamBuf& B, int nt)
{
    if (B.observed == 0) return std::max<size_t>(65536, (size_t)nt * 16);
    return B.observed + B.observed / 4 + 4096;
}

// The widest tile cone: lanes lie within 4 pixels of the reference lane in
// each axis, and on the film plane z = -1 (|d0| >= 1) an angle is at most the
// distance; wave_cone lowers the cosine by 1e-6 (plus < 5e-7 of rounding).
// rt_cb_tiles_boxes checks every tile against it (a wider tile gets no list);
// the launch-camera boxes rely on it analytically, so they are used only
// while the 4-pixel distance itself stays below the 1-radian cap (*uncapped).
static float tile_wbound(const rt_frame* f, float& cos_wbound, bool* uncapped = nullptr)
{
    const double px = 2.0 * f->half_w * (double)f->inv_w, py = 2.0 * f->half_h * (double)f->inv_h;
    const double a = std::sqrt(16.0 * px * px + 16.0 * py * py) * 1.001;
    if (uncapped) *uncapped = a < 1.0;
    const double amax = std::min(1.0, a);
    const double wb = std::acos(std::max(-1.0, std::cos(amax) - 2e-6)) + 1e-6;
    float w = (float)wb;
    if ((double)w < wb) w = std::nextafter(w, INFINITY);
    float cw = (float)std::cos((double)w);
    if ((double)cw < std::cos((double)w)) cw = std::nextafter(cw, INFINITY);
    cos_wbound = cw;
    return w;
}

// The analytic tile cone of the launch-camera path: half-angle wbound as wave_cone holds a cone — cos rounded down,
// sin and chord (+1e-6 like wave_cone) rounded up.  False when the bound is
// capped (wide pixels) or the frame is not a rotation camera (cb_frame_ok).
static bool tile_cone(const rt_frame* f, float& cosW, float& sinW, float& chord)
{
    float cwb = 0.f;
    bool uncapped = false;
    const float wb = tile_wbound(f, cwb, &uncapped);
    const double cw = std::cos((double)wb);
    float cwf = (float)cw;
    if ((double)cwf > cw) cwf = std::nextafter(cwf, -INFINITY);
    const double sw = std::sqrt(std::max(0.0, 1.0 - (double)cwf * cwf)) + 1e-6, ch = std::sqrt(2.0 * (1.0 - cwf)) + 1e-6;
    float swf = (float)sw, chf = (float)ch;
    if ((double)swf < sw) swf = std::nextafter(swf, INFINITY);
    if ((double)chf < ch) chf = std::nextafter(chf, INFINITY);
    cosW = cwf;
    sinW = swf;
    chord = chf;
    return uncapped && cb_frame_ok(f);
}

// ---- camera records in the launch (tiny scenes; rt_cull.h TinyCam)
// Used for depth-0 frames of scenes of 1..kTinyMax triangles whose shadow
// rays go through the light buffer (RT_OPT_LAUNCH_CAMERA, on by default):
// then nothing per camera lives on the device.
static bool tiny_ok(const rt_ctx* c, int depth, bool lbuf)
{
    return c->opt_launch_camera && depth == 0 && lbuf && c->n_tri > 0 && c->n_tri <= kTinyMax &&
           (int)c->h_tri.size() == 3 * c->n_tri;
}

// One mask half-space of rt_cull.h tiny_tile_mask: dot(w, p.xyz) >= p.w,
// the threshold lowered by 1e-6 more than the wave test's margin (the
// device's fused dot product is within 3e-7 of the wave test's) and rounded
// down; a plane with a NaN passes everything, as the wave test's NaN
// comparisons do.
static float4 tiny_plane(const float4 n, double thr)
{
    if (n.x != n.x || n.y != n.y || n.z != n.z || thr != thr) return make_float4(0.f, 0.f, 0.f, -INFINITY);
    thr -= 1e-6;
    float t = (float)thr;
    if ((double)t > thr) t = std::nextafter(t, -INFINITY);
    return make_float4(n.x, n.y, n.z, t);
}

// The frame's camera records (rt_cull.h TinyCam): per triangle the camera
// cone and edge records and the tricam record — the device prepass's own
// functions, in double / float on the host — sorted by (dmin, triangle);
// pairs never reported from this camera (cosT 2) are left out.  Tile masks
// are usable when the orientation is a rotation and the tiles' spread bound
// holds analytically (tile_wbound); the mask pointer is set by tiny_masks.
static void tiny_build(const rt_ctx* c, const rt_frame* f, TinyCam& T)
{
    const int n = c->n_tri;
    float4 cone[kTinyMax * kConeRec], tc[kTinyMax * 4];
    for (int k = 0; k < n; ++k)
        cone_record(c->h_tri.data(), c->h_sph.data(), c->h_nrm.data(), c->h_coef.data(), n, f->cam_pos[0],
                    f->cam_pos[1], f->cam_pos[2], 1, 0.0f, cone, tc, k);
    int ord[kTinyMax], m = 0;
    float key[kTinyMax];
    for (int k = 0; k < n; ++k) {
        if (cone[2 * k].w > 1.0f) continue;  // never reported from this camera
        key[k] = cone[2 * k + 1].x == cone[2 * k + 1].x ? cone[2 * k + 1].x : -INFINITY;
        ord[m++] = k;
    }
    std::sort(ord, ord + m, [&](int a, int b) { return key[a] < key[b] || (key[a] == key[b] && a < b); });
    T = TinyCam{};
    T.n = m;
    float cwf, swf, chf;
    T.masked = tile_cone(f, cwf, swf, chf) ? 1 : 0;
    T.tiles_x = (f->width + 7) / 8;
    T.tiles_y = (f->height + 7) / 8;
    T.cosW = cwf;
    T.sinW = swf;
    T.chord = chf;
    for (int j = 0; j < m; ++j) {
        const int k = ord[j];
        float4* r = T.rec + 8 * j;
        const float4 c0 = cone[2 * k];
        const float sinT = cone[2 * k + 1].w;
        // cone_overlap at ang 0: pass iff !(cosT > 0) or dot(w, axis) >=
        // cosW cosT - sinW sinT - 2e-6
        float4 p[4];
        p[0] = c0.w > 0.0f ? tiny_plane(c0, (double)cwf * c0.w - (double)swf * sinT - 2e-6)
                           : make_float4(0.f, 0.f, 0.f, -INFINITY);
        // edge_open at ang 0: pass iff !(dot(w, e) + chord + 2e-6 < e.w)
        for (int e = 0; e < 3; ++e) {
            const float4 ed = cone[2 * n + 3 * k + e];
            p[1 + e] = tiny_plane(ed, (double)ed.w - (double)chf - 2e-6);
        }
        for (int h = 0; h < 2; ++h) {  // paired for the packed FMAs (TinyLane)
            const float4 u = p[2 * h], v = p[2 * h + 1];
            r[2 * h] = make_float4(u.x, v.x, u.y, v.y);
            r[2 * h + 1] = make_float4(u.z, v.z, u.w, v.w);
        }
        for (int q = 0; q < 4; ++q) r[4 + q] = tc[4 * k + q];
        r[7].z = key[k];
        r[7].w = 0.0f;
    }
}

// The frame's records, cached per camera (the host's part of a moving frame).
static const TinyCam& tiny_prepare(rt_ctx* c, const rt_frame* f)
{
    float key[30];
    cb_key_of(f, key);
    if (!c->tiny_valid || std::memcmp(key, c->tiny_key, sizeof key) != 0) {
        tiny_build(c, f, c->tiny);
        std::memcpy(c->tiny_key, key, sizeof key);
        c->tiny_valid = true;
    }
    return c->tiny;
}

// Tile masks of the launch-camera path (*mode, the trace kernel's: 0 read
// the stream's stored masks, 1 compute them in the kernel, 2 compute and
// store them).  One buffer per stream: launches on one stream run in order,
// so a stream's masks are rewritten only after its earlier renders read
// them.  A camera's first frame on a stream computes its masks without
// storing them — a moving camera never reads them back, and the store cost
// a moving C2 frame 7% (A/B) —, its next frame on the stream computes and
// stores them, its later frames read them.  A hipGraph capture computes them
// (its replays recompute: no buffer).  Sets T.mask.
// Buffers are found by the stream's handle, which a destroyed stream's
// successor may reuse: the storing kernel is followed by an event
// (tiny_masks_stored) that a reader waits for while it has not passed.  At
// most kMaskBufs buffers: the least recently used one is dropped (freed at
// the next host sync).
constexpr size_t kMaskBufs = 16;
static int tiny_masks(rt_ctx* c, const rt_frame* f, hipStream_t st, bool capturing, TinyCam& T, int* mode)
{
    *mode = 0;
    if (!T.masked) return RT_OK;  // every listed triangle
    *mode = 1;
    if (capturing) return RT_OK;
    const size_t nt = (size_t)T.tiles_x * T.tiles_y;
    rt_ctx::MaskBuf* b = nullptr;
    for (auto& q : c->tiny_masks)
        if (q.stream == st) b = &q;
    if (!b) {
        if (c->tiny_masks.size() >= kMaskBufs) {
            auto lru = std::min_element(c->tiny_masks.begin(), c->tiny_masks.end(),
                                        [](const rt_ctx::MaskBuf& x, const rt_ctx::MaskBuf& y) { return x.used < y.used; });
            if (lru->d) free_later(c, lru->d);
            if (lru->ev) HIP_TRY(c, hipEventDestroy(lru->ev));  // (released once it has passed)
            c->tiny_masks.erase(lru);
        }
        c->tiny_masks.push_back(rt_ctx::MaskBuf{});
        b = &c->tiny_masks.back();
        b->stream = st;
    }
    b->used = ++c->mask_clock;
    float key[30];
    cb_key_of(f, key);
    if (b->valid && b->cap >= nt && std::memcmp(key, b->key, sizeof key) == 0) {
        if (b->ev_set) {
            const hipError_t q = hipEventQuery(b->ev);
            if (q == hipErrorNotReady) HIP_TRY(c, hipStreamWaitEvent(st, b->ev, 0));
            else if (q == hipSuccess) b->ev_set = false;
            else return hip_fail(c, q, "hipEventQuery");
        }
        T.mask = b->d;
        *mode = 0;
        return RT_OK;
    }
    if (!b->pend_valid || std::memcmp(key, b->pend, sizeof key) != 0) {
        std::memcpy(b->pend, key, sizeof key);  // a new camera: compute only
        b->pend_valid = true;
        return RT_OK;
    }
    if (b->cap < nt) {  // the camera's second frame: compute and store
        if (b->d) free_later(c, b->d);
        b->d = nullptr;
        b->cap = 0;
        b->valid = false;
        HIP_TRY(c, hipMalloc((void**)&b->d, nt * sizeof(unsigned)));
        b->cap = nt;
    }
    std::memcpy(b->key, key, sizeof key);
    b->valid = true;
    b->pend_valid = false;
    T.mask = b->d;
    *mode = 2;
    return RT_OK;
}

// After the kernel that stored stream st's masks (mode 2): their event.
static int tiny_masks_stored(rt_ctx* c, hipStream_t st)
{
    for (auto& q : c->tiny_masks)
        if (q.stream == st) {
            if (!q.ev) HIP_TRY(c, hipEventCreateWithFlags(&q.ev, hipEventDisableTiming));
            HIP_TRY(c, hipEventRecord(q.ev, st));
            q.ev_set = true;
        }
    return RT_OK;
}

static CbDev cb_dev(const rt_ctx::CamBuf& B, const rt_frame* f)
{
    CbDev d;
    d.tcone = B.tcone;
    d.off = B.off;
    d.cur = B.cur;
    d.flag = B.flag;
    d.ent = B.ent;
    d.box = B.box;
    d.tcnt = B.tcnt;
    d.rmask = B.rmask;
    d.rcap = (unsigned)std::min<size_t>(B.rcap, 0xFFFFFFF0u);
    d.lng = B.lng;
    d.mid = B.mid;
    d.stat = B.stat;
    d.cap = (unsigned)B.cap;
    d.tiles_x = (f->width + 7) / 8;
    d.tiles_y = (f->height + 7) / 8;
    d.wbound = tile_wbound(f, d.cos_wbound);
    return d;
}

// Build the camera buffer B for frame f on stream st, from the per-camera
// cone records in S (S.cone_cam; the tricam records for inline entries).
// No host sync — except with `exact_first` (a synchronous render's first
// build, when no total was ever read back: the count is read once and the
// capacity sized to it before the fill).  Needs st ordered after every render that may read
// B.  capturing: inside a hipGraph capture (no timing events, no read-back).
static int cb_build(rt_ctx* c, rt_ctx::CamBuf& B, const rt_frame* f, const SceneDev& S, hipStream_t st,
                    bool exact_first, bool capturing, bool allow_inline)
{
    const auto t0 = std::chrono::steady_clock::now();
    const int tx = (f->width + 7) / 8, ty = (f->height + 7) / 8, nt = tx * ty;
    B.valid = false;
    if (B.pinned) {
        free_later(c, B.off);
        free_later(c, B.flag);
        free_later(c, B.ent);
        free_later(c, B.rec);
        B.off = B.flag = nullptr;
        B.ent = nullptr;
        B.rec = nullptr;
        B.nt_alloc = 0;  // every per-tile array is reallocated
        B.cap = B.rec_cap = 0;
        B.pinned = false;
    }
    if (!capturing) cb_harvest(B);
    if (int rc = cb_ensure(c, B, nt, capturing)) return rc;
    const size_t fixed = (size_t)c->opt_cb_capacity;  // RT_OPT_CB_CAPACITY (tests)
    exact_first = exact_first && B.observed == 0 && !capturing && !fixed;
    if (fixed && !capturing && B.cap != fixed) {
        free_later(c, B.ent);
        B.ent = nullptr;
        B.cap = 0;
    }
    // no growth inside a capture (the caller checked B.cap > 0)
    const size_t want = capturing ? B.cap : (fixed ? fixed : std::max(B.cap, cb_want_cap(B, nt)));
    if (!exact_first)
        if (int rc = cb_grow(c, B, want)) return rc;
    // Device timing (rt_debug_cb_info) of synchronous builds only: a timing
    // event's record drains the queue, which in an async frame is a gap of
    // several us before and after the build (rocprofv3 timeline, C3).
    const bool timed = !capturing && exact_first;
    if (timed) HIP_TRY(c, hipEventRecord(B.ev0, st));
    FrameDev F;
    frame_dev(f, F);
    CbDev D = cb_dev(B, f);
    const unsigned tb = (unsigned)((nt + 3) / 4);
    constexpr unsigned kPairGrid = 2048, kMidGrid = 2048;
    const bool small = c->n_clu == 0;  // small lists: a tile walk instead of the binning
    unsigned long long* tot = nullptr;
    if (small) {
        hipLaunchKernelGGL(rt_cb_walk<false>, dim3(tb), dim3(256), 0, st, S, F, D);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, scan_u32(B.off, (unsigned)nt, B.off, (unsigned long long*)B.scan, st, &tot));
        if (exact_first) {
            HIP_TRY(c, hipMemcpyAsync(B.h_tot, tot, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
            HIP_TRY(c, hipStreamSynchronize(st));
            B.entries = (size_t)B.h_tot[0];
            B.observed = std::max(B.observed, B.entries);
            if (int rc = cb_grow(c, B, cb_want_cap(B, nt))) return rc;
            D.ent = B.ent;
            D.cap = (unsigned)B.cap;
        }
        hipLaunchKernelGGL(rt_cb_walk<true>, dim3(tb), dim3(256), 0, st, S, F, D);
    } else {
    const unsigned nbb = (unsigned)((c->n_tri + 255) / 256);
    hipLaunchKernelGGL(rt_cb_tiles_boxes, dim3(nbb + tb), dim3(256), 0, st, S, F, D, nbb);
    HIP_TRY(c, hipGetLastError());
    unsigned long long* ptot = nullptr;  // the candidate pairs' 64-bit total
    HIP_TRY(c, scan_u32(B.tcnt, (unsigned)c->n_tri, B.tcnt, (unsigned long long*)B.scan, st, &ptot));
    if (exact_first) {  // the pass masks sized to the candidate pairs (one read back)
        HIP_TRY(c, hipMemcpyAsync(B.h_tot, ptot, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipStreamSynchronize(st));
        // past 2^32 - 1 pairs the pass tests none and flags every tile (the
        // per-wave path): no masks to size, nothing to remember (as cb_harvest)
        const bool over = B.h_tot[0] > 0xFFFFFFFFull;
        const size_t pairs = over ? 0 : (size_t)B.h_tot[0];
        if (!over) B.observed_pairs = std::max(B.observed_pairs, pairs);
        const size_t runs = (pairs + 63) / 64 + 1024;
        if (runs > B.rcap) {
            free_later(c, B.rmask);
            B.rmask = nullptr;
            B.rcap = 0;
            HIP_TRY(c, hipMalloc((void**)&B.rmask, runs * sizeof(unsigned long long)));
            B.rcap = runs;
        }
        D.rmask = B.rmask;
        D.rcap = (unsigned)std::min<size_t>(B.rcap, 0xFFFFFFF0u);
    }
    hipLaunchKernelGGL(rt_cb_pairs<false>, dim3(kPairGrid), dim3(256), 0, st, S, D, (const unsigned long long*)ptot);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, scan_u32(B.off, (unsigned)nt, B.off, (unsigned long long*)B.scan, st, &tot));
    if (exact_first) {  // size the entries to the count (the fill is the only reader of the capacity)
        HIP_TRY(c, hipMemcpyAsync(B.h_tot, tot, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipStreamSynchronize(st));
        B.entries = (size_t)B.h_tot[0];
        B.observed = std::max(B.observed, B.entries);
        if (int rc = cb_grow(c, B, cb_want_cap(B, nt))) return rc;
        D.ent = B.ent;
        D.cap = (unsigned)B.cap;
    }
    hipLaunchKernelGGL(rt_cb_pairs<true>, dim3(kPairGrid), dim3(256), 0, st, S, D, (const unsigned long long*)nullptr);
    }
    hipLaunchKernelGGL(rt_cb_keys_small, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, D, nt);
    hipLaunchKernelGGL(rt_cb_keys_rest, dim3(kMidGrid), dim3(256), 0, st, D, (const unsigned long long*)tot,
                       capturing ? (unsigned long long*)nullptr : B.h_tot);
    HIP_TRY(c, hipGetLastError());
    // inline records while the capacity fits RT_OPT_CB_INLINE_MAX_MB
    B.inline_rec = allow_inline && (double)B.cap * 4 * sizeof(float4) <= c->opt_cb_inline_mb * 1048576.0;
    if (B.inline_rec) {
        if (B.rec_cap < B.cap || !B.rec) {
            free_later(c, B.rec);
            B.rec = nullptr;
            B.rec_cap = 0;
            HIP_TRY(c, hipMalloc((void**)&B.rec, B.cap * 4 * sizeof(float4)));
            B.rec_cap = B.cap;
        }
        hipLaunchKernelGGL(rt_cb_expand, dim3((unsigned)((B.cap + 255) / 256)), dim3(256), 0, st,
                           (const int2*)B.ent, (const unsigned long long*)tot, (unsigned)B.cap,
                           (const float4*)S.tricam, B.rec);
        HIP_TRY(c, hipGetLastError());
    }
    if (!capturing) {
        HIP_TRY(c, hipEventRecord(B.ev_tot, st));  // rt_cb_keys_rest wrote h_tot
        B.tot_pending = true;
        if (timed) HIP_TRY(c, hipEventRecord(B.ev1, st));
        B.timed = timed;
    }
    cb_key_of(f, B.key);
    B.tiles_x = tx;
    B.ntiles = nt;
    B.valid = true;
    B.built_cap = B.cap;
    B.built_rcap = B.rcap;
    B.host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

static bool cb_matches(const rt_ctx::CamBuf& B, const rt_frame* f)
{
    if (!B.valid) return false;
    float key[30];
    cb_key_of(f, key);
    return std::memcmp(key, B.key, sizeof key) == 0;
}

static bool frame_ok(const rt_frame* f)
{
    return !(f->width <= 0 || f->height <= 0 || f->row_begin < 0 || f->row_end > f->height ||
             f->row_begin > f->row_end || f->max_bounces < 0 ||
             (f->band_rows != 0 && rt_band_rows(f->height, f->band_rows, f->band_count, f->band_index) < 0));
}

// Does building a new camera's buffer on the stream pay for an async or
// sequence frame?  Measured (round 3, tools/camera_probe.py, moving camera):
// the build costs ~0.24 ms + 0.017 ms per Mpx (its ~15 launches dominate
// at 1080p), the buffer saves the trace kernel ~0.05-0.09 ms per Mpx of
// per-wave culling on a big list (C3 1080p: 0.418 ms per frame per-wave,
// 0.54 with the build; C5 7680 x 4320: 3.72 per-wave, 3.03 with it); on
// small lists (<= 1,024 triangles) it saves a few us (C2 -3.6%).  So: big
// lists from 4 Mpx of output rows; RT_OPT_CAMERA_BUFFER 2 builds for every
// frame (tests).  Synchronous renders always build (they sync anyway).
static bool cb_async_pays(const rt_ctx* c, const rt_frame* f)
{
    if (c->opt_camera_buffer == 2) return true;
    return c->n_tri > kClusterMinTriangles && (double)f->width * frame_rows(f) >= 4e6;
}

#endif  // RT_AMD_RT_CAMHOST_H
