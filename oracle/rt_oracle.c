/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
 *
 * Plain-C CPU restatement of the Rodyll/Ray-Tracing-GPU hot path (the CPU
 * branch of CScene::LancerRayons and everything it calls), used ONLY by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as
 * the checker / the timed CPU baseline — never as the thing shipped.  The
 * product (ray-tracing-gpu_amd/) never links, loads or calls this file.
 *
 * Parity pinning: this restatement is checked bit-for-bit (float32 RGB) against
 * oracle/_ref/libref_oracle.so, which is built from the reference's OWN
 * primitive / math sources (Triangle.cpp, Plan.cpp, Quadrique.cpp, Matrice4.cpp,
 * Vecteur3.h, Couleur.h, ...) by oracle/Makefile, and against the fixtures in
 * tests/golden/ that the _ref build produced (tests/golden/make_golden.py).
 *
 * All citations are relative to /root/reference/Projet-INF8702/.
 * Arithmetic follows the reference's evaluation order exactly: REAL = float
 * (MathUtils.h:23), no FMA contraction (build with -ffp-contract=off), IEEE
 * division except where the reference multiplies by a reciprocal.
 *
 * Depth > 0: the reference's reflection/refraction block is commented out
 * (Scene.cpp:1779-1823).  oracle_scene.max_bounces == 0 reproduces the shipped
 * executable; > 0 re-enables that block exactly as written ("reference-commented
 * semantics").
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define O_EPS ((float)1.0e-2)             /* MathUtils.h:35 EPSILON            */
#define O_PI ((float)M_PI)                /* MathUtils.h:28-32 RENDRE_REEL(PI) */

/* ------------------------------------------------------------------ Math3D */
typedef struct { float x, y, z; } ov3;
typedef struct { float m[4][4]; } om4;
typedef struct { float r, g, b; } ocol;

static ov3 v3(float x, float y, float z) { ov3 v = {x, y, z}; return v; }
/* Vecteur3.h operator+ / operator- (V1, V2) */
static ov3 v3_add(ov3 a, ov3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static ov3 v3_sub(ov3 a, ov3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static ov3 v3_neg(ov3 a) { return v3(-a.x, -a.y, -a.z); }
/* Vecteur3.h operator*(REAL, V) and (V, REAL): Vecteur.x * Scalaire */
static ov3 v3_mul(ov3 v, float s) { return v3(v.x * s, v.y * s, v.z * s); }
/* Vecteur3.h ProdScal: left to right */
static float v3_dot(ov3 a, ov3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* Vecteur3.h ProdVect */
static ov3 v3_cross(ov3 a, ov3 b)
{
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Vecteur3.h Norme: sqrt(float) -> sqrtf */
static float v3_norme(ov3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
/* Vecteur3.h operator/(REAL): reciprocal then multiply */
static ov3 v3_div(ov3 v, float s)
{
    float inv = 1.0f / s;
    return v3(v.x * inv, v.y * inv, v.z * inv);
}
/* Vecteur3.h Normaliser: ZERO if length <= EPSILON */
static ov3 v3_normaliser(ov3 v)
{
    ov3 r = v3(0.f, 0.f, 0.f);
    float len = v3_norme(v);
    if (len > O_EPS) {
        len = 1.0f / len;
        r = v3_mul(v, len);
    }
    return r;
}
/* Vecteur3.h Reflect: V - (2 * dot(V,N)) * N */
static ov3 v3_reflect(ov3 v, ov3 n)
{
    float s = 2.0f * v3_dot(v, n);
    return v3_sub(v, v3_mul(n, s));
}
/* Vecteur3.h Refract: pow(float,int) promotes to double (C++11 <cmath>),
 * so 1 - |Z|^2 and its sqrt are double; the product with Normal takes REAL. */
static ov3 v3_refract(ov3 v, ov3 n, float eta)
{
    ov3 z = v3_mul(v3_sub(v, v3_mul(n, v3_dot(v, n))), eta);
    double nz = (double)v3_norme(z);
    float s = (float)sqrt(1 - pow(nz, 2));
    ov3 t = v3_sub(z, v3_mul(n, s));
    if (v3_dot(t, n) < 0)
        return t;
    return v3_reflect(v, n);
}

/* Matrice4.h / Matrice4.cpp */
static om4 m4_zero(void) { om4 r; memset(&r, 0, sizeof r); return r; }
static om4 m4_identity(void)
{
    om4 r = m4_zero();
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.0f;
    return r;
}
/* Matrice4.h Concatene: row-by-column, 4 terms left to right */
static om4 m4_concat(const om4* a, const om4* b)
{
    om4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.m[i][j] = a->m[i][0] * b->m[0][j] + a->m[i][1] * b->m[1][j] +
                        a->m[i][2] * b->m[2][j] + a->m[i][3] * b->m[3][j];
    return r;
}
/* Matrice4.h operator*(CVecteur3, CMatrice4): affine point transform */
static ov3 v3_xform(ov3 v, const om4* m)
{
    ov3 r;
    r.x = m->m[0][0] * v.x + m->m[1][0] * v.y + m->m[2][0] * v.z + m->m[3][0];
    r.y = m->m[0][1] * v.x + m->m[1][1] * v.y + m->m[2][1] * v.z + m->m[3][1];
    r.z = m->m[0][2] * v.x + m->m[1][2] * v.y + m->m[2][2] * v.z + m->m[3][2];
    return r;
}
/* Matrice4.cpp:29-106 Inverse (cofactor expansion, same temporaries) */
static om4 m4_inverse(const om4* M)
{
    float m00 = M->m[0][0], m01 = M->m[0][1], m02 = M->m[0][2], m03 = M->m[0][3];
    float m10 = M->m[1][0], m11 = M->m[1][1], m12 = M->m[1][2], m13 = M->m[1][3];
    float m20 = M->m[2][0], m21 = M->m[2][1], m22 = M->m[2][2], m23 = M->m[2][3];
    float m30 = M->m[3][0], m31 = M->m[3][1], m32 = M->m[3][2], m33 = M->m[3][3];
    float v0 = m20 * m31 - m21 * m30;
    float v1 = m20 * m32 - m22 * m30;
    float v2 = m20 * m33 - m23 * m30;
    float v3_ = m21 * m32 - m22 * m31;
    float v4 = m21 * m33 - m23 * m31;
    float v5 = m22 * m33 - m23 * m32;
    float t00 = (v5 * m11 - v4 * m12 + v3_ * m13);
    float t10 = -(v5 * m10 - v2 * m12 + v1 * m13);
    float t20 = (v4 * m10 - v2 * m11 + v0 * m13);
    float t30 = -(v3_ * m10 - v1 * m11 + v0 * m12);
    float invDet = 1.0f / (t00 * m00 + t10 * m01 + t20 * m02 + t30 * m03);
    om4 r;
    r.m[0][0] = t00 * invDet;
    r.m[1][0] = t10 * invDet;
    r.m[2][0] = t20 * invDet;
    r.m[3][0] = t30 * invDet;
    r.m[0][1] = -(v5 * m01 - v4 * m02 + v3_ * m03) * invDet;
    r.m[1][1] = (v5 * m00 - v2 * m02 + v1 * m03) * invDet;
    r.m[2][1] = -(v4 * m00 - v2 * m01 + v0 * m03) * invDet;
    r.m[3][1] = (v3_ * m00 - v1 * m01 + v0 * m02) * invDet;
    v0 = m10 * m31 - m11 * m30;
    v1 = m10 * m32 - m12 * m30;
    v2 = m10 * m33 - m13 * m30;
    v3_ = m11 * m32 - m12 * m31;
    v4 = m11 * m33 - m13 * m31;
    v5 = m12 * m33 - m13 * m32;
    r.m[0][2] = (v5 * m01 - v4 * m02 + v3_ * m03) * invDet;
    r.m[1][2] = -(v5 * m00 - v2 * m02 + v1 * m03) * invDet;
    r.m[2][2] = (v4 * m00 - v2 * m01 + v0 * m03) * invDet;
    r.m[3][2] = -(v3_ * m00 - v1 * m01 + v0 * m02) * invDet;
    v0 = m21 * m10 - m20 * m11;
    v1 = m22 * m10 - m20 * m12;
    v2 = m23 * m10 - m20 * m13;
    v3_ = m22 * m11 - m21 * m12;
    v4 = m23 * m11 - m21 * m13;
    v5 = m23 * m12 - m22 * m13;
    r.m[0][3] = -(v5 * m01 - v4 * m02 + v3_ * m03) * invDet;
    r.m[1][3] = (v5 * m00 - v2 * m02 + v1 * m03) * invDet;
    r.m[2][3] = -(v4 * m00 - v2 * m01 + v0 * m03) * invDet;
    r.m[3][3] = (v3_ * m00 - v1 * m01 + v0 * m02) * invDet;
    return r;
}
static om4 m4_transpose(const om4* a)
{
    om4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r.m[i][j] = a->m[j][i];
    return r;
}
/* Matrice4.h RotationAutourDesX/Y/Z, Translation, MiseAEchelle — all POST:
 * (*this) = Concatene(T).  cos/sin of a float -> cosf/sinf. */
static void m4_post(om4* m, const om4* t) { *m = m4_concat(m, t); }
static void m4_rot_x(om4* m, float rad)
{
    om4 t = m4_identity();
    t.m[1][1] = cosf(rad);
    t.m[1][2] = sinf(rad);
    t.m[2][2] = t.m[1][1];
    t.m[2][1] = -t.m[1][2];
    m4_post(m, &t);
}
static void m4_rot_y(om4* m, float rad)
{
    om4 t = m4_identity();
    t.m[0][0] = cosf(rad);
    t.m[0][2] = -sinf(rad);
    t.m[2][2] = t.m[0][0];
    t.m[2][0] = -t.m[0][2];
    m4_post(m, &t);
}
static void m4_rot_z(om4* m, float rad)
{
    om4 t = m4_identity();
    t.m[0][0] = cosf(rad);
    t.m[0][1] = sinf(rad);
    t.m[1][1] = t.m[0][0];
    t.m[1][0] = -t.m[0][1];
    m4_post(m, &t);
}
static void m4_translate(om4* m, float x, float y, float z)
{
    om4 t = m4_identity();
    t.m[3][0] = x;
    t.m[3][1] = y;
    t.m[3][2] = z;
    m4_post(m, &t);
}
static void m4_scale(om4* m, float x, float y, float z)
{
    om4 t = m4_identity();
    t.m[0][0] = x;
    t.m[1][1] = y;
    t.m[2][2] = z;
    m4_post(m, &t);
}
/* MathUtils.h:132-136 Deg2Rad<float> */
static float deg2rad(float a) { return (a / 180.0f) * O_PI; }

/* Couleur.h: CCouleur(int,int,int) = R * (1.0f/255.0f), no clamp */
static const float UBYTE_2_FLOAT_INIT = 1.0f / 255.0f;
static ocol col_from_int(int r, int g, int b)
{
    ocol c;
    c.r = r * UBYTE_2_FLOAT_INIT;
    c.g = g * UBYTE_2_FLOAT_INIT;
    c.b = b * UBYTE_2_FLOAT_INIT;
    return c;
}
static ocol col_scale(ocol c, float s) { ocol r = {c.r * s, c.g * s, c.b * s}; return r; }
static ocol col_mul(ocol a, ocol b) { ocol r = {a.r * b.r, a.g * b.g, a.b * b.b}; return r; }
static void col_addeq(ocol* a, ocol b) { a->r += b.r; a->g += b.g; a->b += b.b; }
static void col_muleq(ocol* a, ocol b) { a->r *= b.r; a->g *= b.g; a->b *= b.b; }

/* ------------------------------------------------------------ scene model */
enum { O_TRI = 0, O_PLANE = 1, O_QUAD = 2 };

typedef struct {
    int type;
    /* ISurface.h:25-41, defaults ISurface.cpp:15-25 */
    ocol color;
    float ka, kd, ks, shin, kr, kt, ior;
    om4 xf;
    /* Triangle.h m_Pts / m_Normale; Plan.h m_Normale / m_Cst;
     * Quadrique.h m_Quadratique / m_Lineaire / m_Mixte / m_Cst */
    ov3 pts[3];
    ov3 normal;
    ov3 quad, lin, mix;
    float cst;
} osurf;

typedef struct {
    ov3 pos;     /* Lumiere.h m_Position  (default ZERO)   */
    ocol color;  /* m_Couleur   (default BLANC)             */
    float intens;/* m_Intensite (default 0)                 */
} olight;

typedef struct oracle_scene {
    int w, h;
    int max_bounces;      /* Scene.cpp:68 m_NbRebondsMax            */
    float min_energy;     /* Scene.cpp:69 m_EnergieMinRayon = 0.01 */
    float scene_ior;      /* Scene.cpp:70 m_IndiceRefractionScene  */
    ocol background;
    ov3 cam_pos, cam_eye, cam_up;
    float focale, angle;
    om4 orient;
    osurf* surf;
    int nsurf, capsurf;
    olight* lights;
    int nlights, caplights;
    float half_w, half_h, inv_w, inv_h;
    int prepared;
    char err[256];
} oracle_scene;

typedef struct {
    ov3 o, d;
    float ior, energy;
    int bounces;
} oray;

typedef struct {
    int surf;   /* index or -1 */
    float t;    /* Intersection.cpp: default -1 */
    ov3 n;
} ohit;

static void surf_defaults(osurf* s, int type)
{
    memset(s, 0, sizeof *s);
    s->type = type;
    s->color.r = s->color.g = s->color.b = 0.0f; /* CCouleur::NOIR */
    s->ka = 0.2f;
    s->kd = 0.8f;
    s->ks = 0.0f;
    s->shin = 0.0f;
    s->kr = 0.0f;
    s->kt = 0.0f;
    s->ior = 0.0f;
    s->xf = m4_identity();
}

static osurf* push_surf(oracle_scene* s, int type)
{
    if (s->nsurf == s->capsurf) {
        s->capsurf = s->capsurf ? s->capsurf * 2 : 64;
        s->surf = (osurf*)realloc(s->surf, (size_t)s->capsurf * sizeof(osurf));
    }
    osurf* r = &s->surf[s->nsurf++];
    surf_defaults(r, type);
    return r;
}
static olight* push_light(oracle_scene* s)
{
    if (s->nlights == s->caplights) {
        s->caplights = s->caplights ? s->caplights * 2 : 8;
        s->lights = (olight*)realloc(s->lights, (size_t)s->caplights * sizeof(olight));
    }
    olight* l = &s->lights[s->nlights++];
    l->pos = v3(0.f, 0.f, 0.f);
    l->color.r = l->color.g = l->color.b = 1.0f; /* CCouleur::BLANC */
    l->intens = 0.0f;
    return l;
}

/* ----------------------------------------------------------------- parser */
/* Scene.cpp:231-501 CScene::TraiterFichierDeScene.
 * - getline(Line, 80) (Scene.h:86): at most 79 chars; a longer line sets
 *   failbit and the reference's while(!eof()) loop never terminates.  We
 *   report that as an error instead of hanging.
 * - CStringUtils::Trim's result is discarded (Scene.cpp:254), so the buffer is
 *   NOT trimmed: a comment is a line whose FIRST raw char is '*'.
 * - keywords are substring matches (STRING_CHECKFIND, Scene.cpp:39).
 * - R,G,B / Val0..2 are function-scope and keep stale values when a sscanf
 *   conversion fails (reference: uninitialised; here: 0 at start).
 * - Objects are appended in file order when the next object keyword arrives,
 *   and the last one at EOF (lights pushed after surfaces at EOF). */
enum { ST_SCENE, ST_LIGHT, ST_TRI, ST_PLANE, ST_QUAD };
#define HAS(buf, key) (strstr((buf), (key)) != NULL)

static int oracle_parse(oracle_scene* S, const char* path)
{
    FILE* f = fopen(path, "rb");
    if (!f) {
        snprintf(S->err, sizeof S->err, "cannot open %s", path);
        return -1;
    }
    int state = ST_SCENE;
    int cur_surf = -1, cur_light = -1;   /* pending object (not yet pushed) */
    /* pending objects are created directly in the arrays but their order is
     * the push order: surfaces and lights live in separate vectors, so
     * creating at keyword time == pushing at the next keyword. */
    char line[80];
    char tok[80];
    float v0 = 0, v1 = 0, v2 = 0;
    int R = 0, G = 0, B = 0;
    int eof = 0;
    while (!eof) {
        /* istream::getline(line, 80) */
        int n = 0, c;
        for (;;) {
            c = fgetc(f);
            if (c == EOF) { eof = 1; break; }
            if (c == '\n') break;
            if (n == 79) {
                fclose(f);
                snprintf(S->err, sizeof S->err,
                         "line longer than 79 chars in %s (reference getline sets failbit and loops forever)", path);
                return -2;
            }
            line[n++] = (char)c;
        }
        line[n] = 0;
        /* std::string Buffer = Line;  — stops at an embedded NUL like the reference */
        const char* buf = line;
        if (buf[0] == 0 || buf[0] == '*') continue;

        int newobj = 1, nstate = state;
        if (HAS(buf, "Lumiere:")) nstate = ST_LIGHT;
        else if (HAS(buf, "Poly:")) nstate = ST_TRI;
        else if (HAS(buf, "Plane:")) nstate = ST_PLANE;
        else if (HAS(buf, "Quad:")) nstate = ST_QUAD;
        else newobj = 0;

        if (newobj) {
            state = nstate;
            cur_surf = cur_light = -1;
            switch (state) {
            case ST_LIGHT: push_light(S); cur_light = S->nlights - 1; break;
            case ST_TRI: push_surf(S, O_TRI); cur_surf = S->nsurf - 1; break;
            case ST_PLANE: push_surf(S, O_PLANE); cur_surf = S->nsurf - 1; break;
            case ST_QUAD: push_surf(S, O_QUAD); cur_surf = S->nsurf - 1; break;
            }
            continue;
        }
        if (cur_surf >= 0) {
            osurf* s = &S->surf[cur_surf];
            int generic = 1;
            if (HAS(buf, "color:")) {
                sscanf(buf, "%s %i %i %i", tok, &R, &G, &B);
                s->color = col_from_int(R, G, B);
            } else if (HAS(buf, "ambient:")) {
                sscanf(buf, "%s %f", tok, &v0);
                s->ka = v0;
            } else if (HAS(buf, "diffus:")) {
                sscanf(buf, "%s %f", tok, &v0);
                s->kd = v0;
            } else if (HAS(buf, "specular:")) {
                sscanf(buf, "%s %f %f", tok, &v0, &v1);
                s->ks = v0;
                s->shin = v1;
            } else if (HAS(buf, "reflect:")) {
                sscanf(buf, "%s %f", tok, &v0);
                s->kr = v0;
            } else if (HAS(buf, "refract:")) {
                sscanf(buf, "%s %f %f", tok, &v0, &v1);
                s->kt = v0;
                s->ior = v1;
            } else if (HAS(buf, "rotate:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                m4_rot_x(&s->xf, deg2rad(v0));
                m4_rot_y(&s->xf, deg2rad(v1));
                m4_rot_z(&s->xf, deg2rad(v2));
            } else if (HAS(buf, "translate:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                m4_translate(&s->xf, v0, v1, v2);
            } else if (HAS(buf, "scale:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                m4_scale(&s->xf, v0, v1, v2);
            } else
                generic = 0;
            if (generic) continue;
        }
        switch (state) {
        case ST_SCENE:
            if (HAS(buf, "background:")) {
                sscanf(buf, "%s %i %i %i", tok, &R, &G, &B);
                S->background = col_from_int(R, G, B);
            } else if (HAS(buf, "origin:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->cam_pos = v3(v0, v1, v2);
            } else if (HAS(buf, "eye:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->cam_eye = v3(v0, v1, v2);
            } else if (HAS(buf, "up:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->cam_up = v3(v0, v1, v2);
            }
            break;
        case ST_LIGHT: {
            olight* l = &S->lights[cur_light];
            if (HAS(buf, "position:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                l->pos = v3(v0, v1, v2);
            } else if (HAS(buf, "intens:")) {
                sscanf(buf, "%s %f", tok, &v0);
                l->intens = v0;
            } else if (HAS(buf, "color:")) {
                sscanf(buf, "%s %i %i %i", tok, &R, &G, &B);
                l->color = col_from_int(R, G, B);
            }
            break;
        }
        case ST_TRI:
            if (HAS(buf, "point:")) {
                int idx = -1;
                sscanf(buf, "%s %i %f %f %f", tok, &idx, &v0, &v1, &v2);
                if (idx < 0 || idx > 2) { /* Triangle.h:56 assert */
                    fclose(f);
                    snprintf(S->err, sizeof S->err, "triangle point index %d out of range", idx);
                    return -3;
                }
                S->surf[cur_surf].pts[idx] = v3(v0, v1, v2);
            }
            break;
        case ST_PLANE:
            if (HAS(buf, "v_linear:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->surf[cur_surf].normal = v3(v0, v1, v2);
            } else if (HAS(buf, "v_const:")) {
                sscanf(buf, "%s %f", tok, &v0);
                S->surf[cur_surf].cst = v0;
            }
            break;
        case ST_QUAD:
            if (HAS(buf, "v_quad:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->surf[cur_surf].quad = v3(v0, v1, v2);
            } else if (HAS(buf, "v_mixte:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->surf[cur_surf].mix = v3(v0, v1, v2);
            } else if (HAS(buf, "v_linear:")) {
                sscanf(buf, "%s %f %f %f", tok, &v0, &v1, &v2);
                S->surf[cur_surf].lin = v3(v0, v1, v2);
            } else if (HAS(buf, "v_const:")) {
                sscanf(buf, "%s %f", tok, &v0);
                S->surf[cur_surf].cst = v0;
            }
            break;
        }
    }
    fclose(f);
    return 0;
}

/* ----------------------------------------------------------- Pretraitement */
/* Triangle.cpp:108-113 + CalculerNormale :199-204 */
static void pre_tri(osurf* s)
{
    for (int i = 0; i < 3; i++) s->pts[i] = v3_xform(s->pts[i], &s->xf);
    ov3 e1 = v3_sub(s->pts[1], s->pts[0]);
    ov3 e2 = v3_sub(s->pts[2], s->pts[0]);
    s->normal = v3_normaliser(v3_cross(e1, e2));
}
/* Plan.cpp:101-114 (the translation row also moves the normal) */
static void pre_plane(osurf* s)
{
    s->normal = v3_normaliser(v3_xform(s->normal, &s->xf));
    float pt[3] = {0.f, 0.f, 0.f};
    float nn[3] = {s->normal.x, s->normal.y, s->normal.z};
    for (int i = 0; i < 3; i++)
        if (nn[i] != 0) pt[i] = -(s->cst / nn[i]);
    ov3 p = v3_xform(v3(pt[0], pt[1], pt[2]), &s->xf);
    s->cst = v3_dot(v3_neg(s->normal), p);
}
/* Quadrique.cpp:110-146 (Goldman: Q' = M^-1 Q M^-T) */
static void pre_quad(osurf* s)
{
    float A = s->quad.x, B = s->quad.y, C = s->quad.z;
    float D = s->mix.z * 0.5f, E = s->mix.x * 0.5f, F = s->mix.y * 0.5f;
    float G = s->lin.x * 0.5f, H = s->lin.y * 0.5f, J = s->lin.z * 0.5f;
    float K = s->cst;
    om4 Q = {{{A, D, F, G}, {D, B, E, H}, {F, E, C, J}, {G, H, J, K}}};
    om4 inv = m4_inverse(&s->xf);
    om4 invT = m4_transpose(&inv);
    om4 t = m4_concat(&inv, &Q);
    Q = m4_concat(&t, &invT);
    s->quad = v3(Q.m[0][0], Q.m[1][1], Q.m[2][2]);
    s->cst = Q.m[3][3];
    s->mix = v3(Q.m[1][2] * 2.0f, Q.m[0][2] * 2.0f, Q.m[0][1] * 2.0f);
    s->lin = v3(Q.m[0][3] * 2.0f, Q.m[1][3] * 2.0f, Q.m[2][3] * 2.0f);
}

/* Scene.cpp:624-660 InitialiserCamera (libm: atan2 of floats -> atan2f) */
static void init_camera(oracle_scene* S)
{
    const float DIM_FILM_CAM = 0.024f;           /* Scene.cpp:42 */
    float d2 = v3_norme(v3_sub(S->cam_pos, S->cam_eye));
    float y2 = (d2 / (S->focale * 0.001f) - 1) * DIM_FILM_CAM;
    S->angle = (360 * atan2f(y2 * 0.5f, d2)) / O_PI;
    ov3 N = v3_normaliser(v3_sub(S->cam_pos, S->cam_eye));
    ov3 V = v3_normaliser(v3_sub(S->cam_up, v3_mul(N, v3_dot(S->cam_up, N))));
    ov3 U = v3_cross(V, N);
    om4 o = {{{U.x, U.y, U.z, 0.0f}, {V.x, V.y, V.z, 0.0f}, {N.x, N.y, N.z, 0.0f}, {0.0f, 0.0f, 0.0f, 1.0f}}};
    S->orient = o;
}

/* ---------------------------------------------------------- intersections */
/* Triangle.cpp:127-172 (Moller-Trumbore, edges recomputed per test) */
static ohit isect_tri(const osurf* s, int idx, const oray* r)
{
    ohit h = {-1, -1.0f, {0, 0, 0}};
    ov3 e1 = v3_sub(s->pts[1], s->pts[0]);
    ov3 e2 = v3_sub(s->pts[2], s->pts[0]);
    ov3 p = v3_cross(r->d, e2);
    float det = v3_dot(e1, p);
    float adet = det > 0 ? det : -det;   /* MathUtils.h Abs */
    if (adet < O_EPS) return h;
    float inv = 1.0f / det;
    ov3 sv = v3_sub(r->o, s->pts[0]);
    float u = v3_dot(sv, p) * inv;
    if (u < 0 || u > 1) return h;
    ov3 q = v3_cross(sv, e1);
    float v = v3_dot(r->d, q) * inv;
    if (v < 0 || u + v > 1) return h;
    h.surf = idx;
    h.t = v3_dot(e2, q) * inv;
    h.n = s->normal;
    return h;
}
/* Plan.cpp:128-144 */
static ohit isect_plane(const osurf* s, int idx, const oray* r)
{
    ohit h = {-1, -1.0f, {0, 0, 0}};
    float vd = v3_dot(s->normal, r->d);
    float avd = vd > 0 ? vd : -vd;
    if (avd > O_EPS) {
        h.surf = idx;
        h.t = -(v3_dot(s->normal, r->o) + s->cst) / vd;
        h.n = s->normal;
    }
    return h;
}
/* Quadrique.cpp:160-249 (Haines-Heckbert) */
static ohit isect_quad(const osurf* s, int idx, const oray* r)
{
    ohit h = {-1, -1.0f, {0, 0, 0}};
    ov3 d = r->d, o = r->o;
    ov3 q = s->quad, m = s->mix, l = s->lin;
    const float A = d.x * (q.x * d.x + m.z * d.y + m.y * d.z) +
                    d.y * (q.y * d.y + m.x * d.z) +
                    d.z * (q.z * d.z);
    const float Bc = d.x * (q.x * o.x + 0.5f * (m.z * o.y + m.y * o.z + l.x)) +
                     d.y * (q.y * o.y + 0.5f * (m.z * o.x + m.x * o.z + l.y)) +
                     d.z * (q.z * o.z + 0.5f * (m.y * o.x + m.x * o.y + l.z));
    const float Cc = o.x * (q.x * o.x + m.z * o.y + m.y * o.z + l.x) +
                     o.y * (q.y * o.y + m.x * o.z + l.y) +
                     o.z * (q.z * o.z + l.z) +
                     s->cst;
    if (A != 0.0) {
        float Ka = -Bc / A;
        float Kb = Cc / A;
        float delta = Ka * Ka - Kb;
        if (delta > 0) {
            delta = sqrtf(delta);
            float t0 = Ka - delta;
            float t1 = Ka + delta;
            float dist = t0 < t1 ? t0 : t1;           /* Min<REAL> */
            if (dist < O_EPS) dist = t0 > t1 ? t0 : t1; /* Max<REAL> */
            if (!(dist < 0)) {
                h.t = dist;
                h.surf = idx;
                ov3 hp = v3_add(o, v3_mul(d, dist));
                ov3 n;
                n.x = 2.0f * q.x * hp.x + m.y * hp.z + m.z * hp.y + l.x;
                n.y = 2.0f * q.y * hp.y + m.x * hp.z + m.z * hp.x + l.y;
                n.z = 2.0f * q.z * hp.z + m.x * hp.y + m.y * hp.x + l.z;
                h.n = v3_normaliser(n);
            }
        }
    } else {
        h.surf = idx;
        h.t = -0.5f * (Cc / Bc);
        h.n = v3_normaliser(l);
    }
    return h;
}
static ohit isect(const oracle_scene* S, int i, const oray* r)
{
    const osurf* s = &S->surf[i];
    switch (s->type) {
    case O_TRI: return isect_tri(s, i, r);
    case O_PLANE: return isect_plane(s, i, r);
    default: return isect_quad(s, i, r);
    }
}

/* ----------------------------------------------------------------- shading */
static ocol obtenir_couleur(const oracle_scene* S, const oray* r);

/* Scene.cpp:1842-1861 ObtenirFiltreDeSurface (normalises the ray IN PLACE) */
static ocol filtre(const oracle_scene* S, oray* lr)
{
    ocol F = {1.0f, 1.0f, 1.0f};
    float dist = v3_norme(lr->d);
    lr->d = v3_div(lr->d, dist);
    for (int i = 0; i < S->nsurf; i++) {
        ohit h = isect(S, i, lr);
        if (h.t > O_EPS && h.t < dist)
            col_muleq(&F, col_scale(S->surf[h.surf].color, S->surf[h.surf].kt));
    }
    return F;
}

/* Scene.cpp:1740-1826 ObtenirCouleurSurIntersection (+ commented :1779-1823) */
static ocol shade(const oracle_scene* S, const oray* r, const ohit* h)
{
    const osurf* s = &S->surf[h->surf];
    ocol res = col_scale(s->color, s->ka);
    ov3 P = v3_add(r->o, v3_mul(r->d, h->t));
    for (int li = 0; li < S->nlights; li++) {
        const olight* L = &S->lights[li];
        oray lr;
        lr.o = P;
        lr.d = v3_sub(L->pos, P);
        lr.energy = 1;
        lr.ior = 1;
        lr.bounces = 0;
        if (v3_dot(lr.d, h->n) > 0) {
            ocol F = filtre(S, &lr);
            ocol LC = col_mul(L->color, F);
            float g = L->intens * s->kd * v3_dot(h->n, lr.d);
            col_addeq(&res, col_mul(col_scale(s->color, g), LC));
            ov3 rf = v3_reflect(lr.d, h->n);
            float ps = v3_dot(rf, r->d);
            if (ps > 0) {
                float pf = L->intens * s->ks * powf(ps, s->shin);
                col_addeq(&res, col_scale(LC, pf));
            }
        }
    }
    /* reflection (Scene.cpp:1779-1788, commented in the reference) */
    float er = s->kr * r->energy;
    if (er > S->min_energy && r->bounces < S->max_bounces) {
        oray c;
        c.d = v3_reflect(r->d, h->n);
        c.o = P;
        c.energy = er;
        c.bounces = r->bounces + 1;
        c.ior = 0.0f; /* CRayon default, never set for the reflected ray */
        col_addeq(&res, col_scale(obtenir_couleur(S, &c), s->kr));
    }
    /* refraction (Scene.cpp:1790-1823, commented in the reference) */
    float et = s->kt * r->energy;
    if (et > S->min_energy && r->bounces < S->max_bounces) {
        float ratio;
        oray c;
        ov3 n = h->n;
        if (r->ior == s->ior) {
            c.ior = S->scene_ior;
            ratio = s->ior / S->scene_ior;
            n = v3_neg(n);
        } else {
            c.ior = s->ior;
            ratio = S->scene_ior / s->ior;
        }
        c.o = P;
        c.energy = et;
        c.bounces = r->bounces + 1;
        c.d = v3_refract(r->d, n, ratio);
        col_addeq(&res, col_scale(obtenir_couleur(S, &c), s->kt));
    }
    return res;
}

/* Scene.cpp:1705-1720 ObtenirCouleur: closest hit in file order, strict < */
static ocol obtenir_couleur(const oracle_scene* S, const oray* r)
{
    ohit best = {-1, -1.0f, {0, 0, 0}};
    for (int i = 0; i < S->nsurf; i++) {
        ohit h = isect(S, i, r);
        if (h.t > O_EPS && (h.t < best.t || best.t < 0)) best = h;
    }
    if (best.t < 0) return S->background;
    return shade(S, r, &best);
}

/* ------------------------------------------------------------ public API */
#define OEXPORT __attribute__((visibility("default")))

OEXPORT const char* oracle_error(oracle_scene* S) { return S ? S->err : "null scene"; }

/* CScene ctor (Scene.cpp:44-59) + AjusterResolution + TraiterFichierDeScene
 * + Initialiser (Scene.cpp:140-147: camera, Pretraitement in file order)
 * + the LancerRayons prologue (Scene.cpp:676-679). */
OEXPORT int oracle_load(const char* path, int w, int h, int max_bounces, oracle_scene** out)
{
    oracle_scene* S = (oracle_scene*)calloc(1, sizeof *S);
    *out = S;
    S->w = w;
    S->h = h;
    S->max_bounces = max_bounces;
    S->min_energy = 0.01f;
    S->scene_ior = 1.0f;
    S->background.r = S->background.g = S->background.b = 0.0f;
    S->cam_up = v3(0.f, 1.f, 0.f);
    S->focale = 50.0f;
    S->orient = m4_identity();
    int rc = oracle_parse(S, path);
    if (rc) return rc;
    if (w <= 0 || h <= 0) {
        snprintf(S->err, sizeof S->err, "bad resolution %dx%d", w, h);
        return -4;
    }
    init_camera(S);
    for (int i = 0; i < S->nsurf; i++) {
        switch (S->surf[i].type) {
        case O_TRI: pre_tri(&S->surf[i]); break;
        case O_PLANE: pre_plane(&S->surf[i]); break;
        default: pre_quad(&S->surf[i]); break;
        }
    }
    S->half_h = tanf(deg2rad(S->angle * 0.5f));
    S->half_w = ((float)S->w / S->h) * S->half_h;
    S->inv_w = 1.0f / S->w;
    S->inv_h = 1.0f / S->h;
    S->prepared = 1;
    return 0;
}

OEXPORT void oracle_set_params(oracle_scene* S, int max_bounces, float min_energy, float scene_ior)
{
    S->max_bounces = max_bounces;
    S->min_energy = min_energy;
    S->scene_ior = scene_ior;
}

/* An explicit camera (the product's rt_frame fields): position, orientation
 * m[i][j] row-major, film half extents, pixel reciprocals and resolution —
 * the state the pixel loop reads (Scene.cpp:1538-1561 with :676-679), as a
 * caller moving the camera between frames sets it (Main.cpp:229-250). */
OEXPORT int oracle_set_camera(oracle_scene* S, const float* pos, const float* orient, float half_w, float half_h,
                              float inv_w, float inv_h, int w, int h)
{
    if (!S || !S->prepared || w <= 0 || h <= 0) return -1;
    S->cam_pos = v3(pos[0], pos[1], pos[2]);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) S->orient.m[i][j] = orient[4 * i + j];
    S->half_w = half_w;
    S->half_h = half_h;
    S->inv_w = inv_w;
    S->inv_h = inv_h;
    S->w = w;
    S->h = h;
    return 0;
}

OEXPORT void oracle_free(oracle_scene* S)
{
    if (!S) return;
    free(S->surf);
    free(S->lights);
    free(S);
}

/* One pixel of the CPU loop (Scene.cpp:1538-1561). */
static ocol pixel(const oracle_scene* S, int px, int py)
{
    oray r;
    r.o = S->cam_pos;
    ov3 d = v3((2 * px * S->inv_w - 1) * S->half_w, (2 * py * S->inv_h - 1) * S->half_h, -1);
    r.d = v3_normaliser(v3_xform(d, &S->orient));
    r.energy = 1;
    r.bounces = 0;
    r.ior = 1;
    return obtenir_couleur(S, &r);
}

/* Renders rows [row0,row1) × cols [col0,col1) into rgb (row-major over the
 * requested window, 3 floats per pixel, row 0 = bottom like m_InfoPixel).
 * nthreads > 1 uses OpenMP over rows (dynamic schedule). */
OEXPORT int oracle_render_window(oracle_scene* S, int row0, int row1, int col0, int col1,
                                 float* rgb, int nthreads)
{
    if (!S || !S->prepared) return -1;
    if (row0 < 0 || row1 > S->h || row0 > row1 || col0 < 0 || col1 > S->w || col0 > col1) return -2;
    int ww = col1 - col0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int y = row0; y < row1; y++) {
        for (int x = col0; x < col1; x++) {
            ocol c = pixel(S, x, y);
            float* o = rgb + ((size_t)(y - row0) * ww + (x - col0)) * 3;
            o[0] = c.r;
            o[1] = c.g;
            o[2] = c.b;
        }
    }
    (void)nthreads;
    return 0;
}

OEXPORT int oracle_render(oracle_scene* S, float* rgb, int nthreads)
{
    return oracle_render_window(S, 0, S->h, 0, S->w, rgb, nthreads);
}

/* Canonical dump of the prepared state (used to pin the product's host loader).
 * Layout per surface (ORACLE_SURF_WORDS floats):
 *   [0] type  [1..3] colour  [4] Ka [5] Kd [6] Ks [7] shin [8] Kr [9] Kt [10] ior
 *   tri  : [11..19] p0 p1 p2   [20..22] normal
 *   plane: [11..13] normal     [14] cst
 *   quad : [11..13] quad [14..16] lin [17..19] mix [20] cst
 * Camera (ORACLE_CAM_WORDS): pos(3) orient(16) angle halfW halfH invW invH bg(3)
 * Light (ORACLE_LIGHT_WORDS): pos(3) colour(3) intensity */
#define ORACLE_SURF_WORDS 24
#define ORACLE_CAM_WORDS 27
#define ORACLE_LIGHT_WORDS 7
OEXPORT int oracle_counts(oracle_scene* S, int* nsurf, int* nlights)
{
    *nsurf = S->nsurf;
    *nlights = S->nlights;
    return 0;
}
OEXPORT int oracle_dump(oracle_scene* S, float* surf, float* cam, float* lights)
{
    for (int i = 0; i < S->nsurf; i++) {
        const osurf* s = &S->surf[i];
        float* o = surf + (size_t)i * ORACLE_SURF_WORDS;
        memset(o, 0, ORACLE_SURF_WORDS * sizeof(float));
        o[0] = (float)s->type;
        o[1] = s->color.r; o[2] = s->color.g; o[3] = s->color.b;
        o[4] = s->ka; o[5] = s->kd; o[6] = s->ks; o[7] = s->shin;
        o[8] = s->kr; o[9] = s->kt; o[10] = s->ior;
        if (s->type == O_TRI) {
            for (int k = 0; k < 3; k++) {
                o[11 + 3 * k] = s->pts[k].x; o[12 + 3 * k] = s->pts[k].y; o[13 + 3 * k] = s->pts[k].z;
            }
            o[20] = s->normal.x; o[21] = s->normal.y; o[22] = s->normal.z;
        } else if (s->type == O_PLANE) {
            o[11] = s->normal.x; o[12] = s->normal.y; o[13] = s->normal.z; o[14] = s->cst;
        } else {
            o[11] = s->quad.x; o[12] = s->quad.y; o[13] = s->quad.z;
            o[14] = s->lin.x; o[15] = s->lin.y; o[16] = s->lin.z;
            o[17] = s->mix.x; o[18] = s->mix.y; o[19] = s->mix.z;
            o[20] = s->cst;
        }
    }
    cam[0] = S->cam_pos.x; cam[1] = S->cam_pos.y; cam[2] = S->cam_pos.z;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) cam[3 + 4 * i + j] = S->orient.m[i][j];
    cam[19] = S->angle; cam[20] = S->half_w; cam[21] = S->half_h;
    cam[22] = S->inv_w; cam[23] = S->inv_h;
    cam[24] = S->background.r; cam[25] = S->background.g; cam[26] = S->background.b;
    for (int i = 0; i < S->nlights; i++) {
        float* o = lights + (size_t)i * ORACLE_LIGHT_WORDS;
        o[0] = S->lights[i].pos.x; o[1] = S->lights[i].pos.y; o[2] = S->lights[i].pos.z;
        o[3] = S->lights[i].color.r; o[4] = S->lights[i].color.g; o[5] = S->lights[i].color.b;
        o[6] = S->lights[i].intens;
    }
    return 0;
}

/* Per-primitive known-answer entry: geometry in the post-Pretraitement layout
 * of oracle_dump words [11..22]; returns 1 on a reported intersection. */
OEXPORT int oracle_intersect(int type, const float* geom, const float* ro, const float* rd,
                             float* t_out, float* n_out)
{
    osurf s;
    surf_defaults(&s, type);
    if (type == O_TRI) {
        for (int k = 0; k < 3; k++) s.pts[k] = v3(geom[3 * k], geom[3 * k + 1], geom[3 * k + 2]);
        s.normal = v3(geom[9], geom[10], geom[11]);
    } else if (type == O_PLANE) {
        s.normal = v3(geom[0], geom[1], geom[2]);
        s.cst = geom[3];
    } else {
        s.quad = v3(geom[0], geom[1], geom[2]);
        s.lin = v3(geom[3], geom[4], geom[5]);
        s.mix = v3(geom[6], geom[7], geom[8]);
        s.cst = geom[9];
    }
    oray r;
    r.o = v3(ro[0], ro[1], ro[2]);
    r.d = v3(rd[0], rd[1], rd[2]);
    r.ior = 1; r.energy = 1; r.bounces = 0;
    ohit h;
    if (type == O_TRI) h = isect_tri(&s, 0, &r);
    else if (type == O_PLANE) h = isect_plane(&s, 0, &r);
    else h = isect_quad(&s, 0, &r);
    *t_out = h.t;
    n_out[0] = h.n.x; n_out[1] = h.n.y; n_out[2] = h.n.z;
    return h.surf >= 0;
}
