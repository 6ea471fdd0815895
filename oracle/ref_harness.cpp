// ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.
//
// Harness around the reference's OWN compiled sources.  oracle/Makefile
// compiles, straight from /root/reference/Projet-INF8702 (never copied):
//   Triangle.cpp Plan.cpp Quadrique.cpp ISurface.cpp Intersection.cpp
//   Rayon.cpp Lumiere.cpp Couleur.cpp Matrice4.cpp Vecteur3.cpp
// together with this file into oracle/_ref/libref_oracle.so.  Every
// intersection, Pretraitement, vector/matrix/colour operator, Reflect and
// Refract executed here is the reference's own code.
//
// Scene.cpp itself is NOT buildable without stand-ins (it includes "Math.h",
// which does not exist on a case-sensitive filesystem, plus GL/GLEW calls with
// no library in the image), so the CScene orchestration it contains —
// TraiterFichierDeScene (Scene.cpp:231-501), InitialiserCamera (:624-660),
// the CPU pixel loop (:1538-1561), ObtenirCouleur (:1705-1720),
// ObtenirCouleurSurIntersection (:1740-1826, with the commented :1779-1823
// block re-enabled when max_bounces > 0) and ObtenirFiltreDeSurface
// (:1842-1861) — is restated below line by line on top of the reference's
// classes.  It uses the same operator expressions, so the arithmetic is the
// reference's.
#include <cstring>
#include <cstdio>
#include <cmath>
#include <fstream>
#include <string>
#include <vector>

#include "Triangle.h"
#include "Plan.h"
#include "Quadrique.h"
#include "Lumiere.h"
#include "Rayon.h"
#include "Intersection.h"
#include "Couleur.h"

using namespace Scene;
using namespace Math3D;

#define REXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct RefScene {
    int ResLargeur = 0, ResHauteur = 0;
    CCouleur CouleurArrierePlan = CCouleur::NOIR;
    int NbRebondsMax = 20;
    REAL EnergieMinRayon = RENDRE_REEL(0.01);
    REAL IndiceRefractionScene = RENDRE_REEL(1.0);
    struct {
        CVecteur3 Position = CVecteur3::ZERO;
        CVecteur3 PointVise = CVecteur3::ZERO;
        CVecteur3 Up = CVecteur3::UNIT_Y;
        CMatrice4 Orientation = CMatrice4::IDENTITE;
        REAL Focale = RENDRE_REEL(50.0);
        REAL Angle = 0;
    } Camera;
    std::vector<ISurface*> Surfaces;
    std::vector<int> Types;  // 0 tri, 1 plane, 2 quad
    std::vector<CLumiere*> Lumieres;
    REAL HalfH = 0, HalfW = 0, InvW = 0, InvH = 0;
    std::string err;

    ~RefScene()
    {
        for (auto* s : Surfaces) delete s;
        for (auto* l : Lumieres) delete l;
    }

    // Scene.cpp:231-501
    int Traiter(const char* Fichier)
    {
        enum { SC, LU, TR, PL, QU };
        std::fstream F(Fichier, std::ios::in);
        if (!F.is_open()) {
            err = "cannot open";
            return -1;
        }
        int Etat = SC;
        char Line[80];
        std::string Buffer;
        CLumiere* Lumiere = nullptr;
        ISurface* Surface = nullptr;
        int SurfaceType = -1;
        float Val0 = 0, Val1 = 0, Val2 = 0;
        int R = 0, G = 0, B = 0;
        while (!F.eof()) {
            F.getline(Line, 80);
            if (F.fail() && !F.eof()) {
                err = "line longer than 79 characters (reference would loop forever)";
                return -2;
            }
            Buffer = Line;
            // CStringUtils::Trim(Buffer, " ") — result discarded in the reference
            if (Buffer.empty() || Buffer[0] == '*') continue;
            bool Nouveau = true;
            int EtatNouveau = Etat;
            if (Buffer.find("Lumiere:") != std::string::npos) EtatNouveau = LU;
            else if (Buffer.find("Poly:") != std::string::npos) EtatNouveau = TR;
            else if (Buffer.find("Plane:") != std::string::npos) EtatNouveau = PL;
            else if (Buffer.find("Quad:") != std::string::npos) EtatNouveau = QU;
            else Nouveau = false;
            if (Nouveau) {
                if (Etat != SC) {
                    if (Etat == LU) Lumieres.push_back(Lumiere);
                    else { Surfaces.push_back(Surface); Types.push_back(SurfaceType); }
                    Surface = nullptr;
                    Lumiere = nullptr;
                }
                Etat = EtatNouveau;
                switch (Etat) {
                case LU: Lumiere = new CLumiere(); break;
                case TR: Surface = new CTriangle(); SurfaceType = 0; break;
                case PL: Surface = new CPlan(); SurfaceType = 1; break;
                case QU: Surface = new CQuadrique(); SurfaceType = 2; break;
                }
                continue;
            }
            auto has = [&](const char* k) { return Buffer.find(k) != std::string::npos; };
            const char* b = Buffer.c_str();
            if (Surface != nullptr) {
                bool Generic = true;
                if (has("color:")) {
                    sscanf(b, "%s %i %i %i", Line, &R, &G, &B);
                    Surface->AjusterCouleur(CCouleur(R, G, B));
                } else if (has("ambient:")) {
                    sscanf(b, "%s %f", Line, &Val0);
                    Surface->AjusterCoeffAmbiant(Val0);
                } else if (has("diffus:")) {
                    sscanf(b, "%s %f", Line, &Val0);
                    Surface->AjusterCoeffDiffus(Val0);
                } else if (has("specular:")) {
                    sscanf(b, "%s %f %f", Line, &Val0, &Val1);
                    Surface->AjusterCoeffSpeculaire(Val0);
                    Surface->AjusterCoeffBrillance(Val1);
                } else if (has("reflect:")) {
                    sscanf(b, "%s %f", Line, &Val0);
                    Surface->AjusterCoeffReflexion(Val0);
                } else if (has("refract:")) {
                    sscanf(b, "%s %f %f", Line, &Val0, &Val1);
                    Surface->AjusterCoeffRefraction(Val0);
                    Surface->AjusterIndiceRefraction(Val1);
                } else if (has("rotate:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    CMatrice4 T = Surface->ObtenirTransformation();
                    T.RotationAutourDesX(Deg2Rad<REAL>(Val0));
                    T.RotationAutourDesY(Deg2Rad<REAL>(Val1));
                    T.RotationAutourDesZ(Deg2Rad<REAL>(Val2));
                    Surface->AjusterTransformation(T);
                } else if (has("translate:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    CMatrice4 T = Surface->ObtenirTransformation();
                    T.Translation(Val0, Val1, Val2);
                    Surface->AjusterTransformation(T);
                } else if (has("scale:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    CMatrice4 T = Surface->ObtenirTransformation();
                    T.MiseAEchelle(Val0, Val1, Val2);
                    Surface->AjusterTransformation(T);
                } else
                    Generic = false;
                if (Generic) continue;
            }
            switch (Etat) {
            case SC:
                if (has("background:")) {
                    sscanf(b, "%s %i %i %i", Line, &R, &G, &B);
                    CouleurArrierePlan = CCouleur(R, G, B);
                } else if (has("origin:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    Camera.Position = CVecteur3(Val0, Val1, Val2);
                } else if (has("eye:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    Camera.PointVise = CVecteur3(Val0, Val1, Val2);
                } else if (has("up:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    Camera.Up = CVecteur3(Val0, Val1, Val2);
                }
                break;
            case LU:
                if (has("position:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    Lumiere->SetPosition(CVecteur3(Val0, Val1, Val2));
                } else if (has("intens:")) {
                    sscanf(b, "%s %f", Line, &Val0);
                    Lumiere->SetIntensity(Val0);
                } else if (has("color:")) {
                    sscanf(b, "%s %i %i %i", Line, &R, &G, &B);
                    Lumiere->AjusterCouleur(CCouleur(R, G, B));
                }
                break;
            case TR:
                if (has("point:")) {
                    int PtIdx = -1;
                    sscanf(b, "%s %i %f %f %f", Line, &PtIdx, &Val0, &Val1, &Val2);
                    if (PtIdx < 0 || PtIdx > 2) {
                        err = "triangle point index out of range";
                        return -3;
                    }
                    ((CTriangle*)Surface)->AjusterPoint(PtIdx, CVecteur3(Val0, Val1, Val2));
                }
                break;
            case PL:
                if (has("v_linear:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    ((CPlan*)Surface)->AjusterNormale(CVecteur3(Val0, Val1, Val2));
                } else if (has("v_const:")) {
                    sscanf(b, "%s %f", Line, &Val0);
                    ((CPlan*)Surface)->AjusterConstante(Val0);
                }
                break;
            case QU:
                if (has("v_quad:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    ((CQuadrique*)Surface)->AjusterQuadratique(CVecteur3(Val0, Val1, Val2));
                } else if (has("v_mixte:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    ((CQuadrique*)Surface)->AjusterMixte(CVecteur3(Val0, Val1, Val2));
                } else if (has("v_linear:")) {
                    sscanf(b, "%s %f %f %f", Line, &Val0, &Val1, &Val2);
                    ((CQuadrique*)Surface)->AjusterLineaire(CVecteur3(Val0, Val1, Val2));
                } else if (has("v_const:")) {
                    sscanf(b, "%s %f", Line, &Val0);
                    ((CQuadrique*)Surface)->AjusterConstante(Val0);
                }
                break;
            }
        }
        if (Surface != nullptr) { Surfaces.push_back(Surface); Types.push_back(SurfaceType); }
        if (Lumiere != nullptr) Lumieres.push_back(Lumiere);
        return 0;
    }

    // Scene.cpp:624-660
    void InitialiserCamera()
    {
        const REAL DIM_FILM_CAM = 0.024f;
        REAL d2 = CVecteur3::Distance(Camera.Position, Camera.PointVise);
        REAL y2 = (d2 / (Camera.Focale * RENDRE_REEL(0.001)) - 1) * DIM_FILM_CAM;
        Camera.Angle = (360 * atan2(y2 * RENDRE_REEL(0.5), d2)) / RENDRE_REEL(PI);
        CVecteur3 N = CVecteur3::Normaliser(Camera.Position - Camera.PointVise);
        CVecteur3 V = CVecteur3::Normaliser(Camera.Up - N * CVecteur3::ProdScal(Camera.Up, N));
        CVecteur3 U = CVecteur3::ProdVect(V, N);
        Camera.Orientation = CMatrice4(U.x, U.y, U.z, 0.0f, V.x, V.y, V.z, 0.0f, N.x, N.y, N.z, 0.0f,
                                       0.0f, 0.0f, 0.0f, 1.0f);
    }

    // Scene.cpp:140-147 + :674-679
    void Initialiser()
    {
        InitialiserCamera();
        for (auto* s : Surfaces) s->Pretraitement();
        HalfH = tan(Deg2Rad<REAL>(Camera.Angle * RENDRE_REEL(0.5)));
        HalfW = (RENDRE_REEL(ResLargeur) / ResHauteur) * HalfH;
        InvW = RENDRE_REEL(1.0) / ResLargeur;
        InvH = RENDRE_REEL(1.0) / ResHauteur;
    }

    // Scene.cpp:1705-1720
    CCouleur ObtenirCouleur(const CRayon& Rayon) const
    {
        CIntersection Result;
        CIntersection Tmp;
        for (auto* s : Surfaces) {
            Tmp = s->Intersection(Rayon);
            if (Tmp.ObtenirDistance() > EPSILON &&
                (Tmp.ObtenirDistance() < Result.ObtenirDistance() || Result.ObtenirDistance() < 0))
                Result = Tmp;
        }
        return (Result.ObtenirDistance() < 0) ? CouleurArrierePlan : ObtenirCouleurSurIntersection(Rayon, Result);
    }

    // Scene.cpp:1740-1826 (commented block :1779-1823 re-enabled)
    CCouleur ObtenirCouleurSurIntersection(const CRayon& Rayon, const CIntersection& I) const
    {
        CCouleur Result = I.ObtenirSurface()->ObtenirCouleur() * I.ObtenirSurface()->ObtenirCoeffAmbiant();
        CVecteur3 P = Rayon.ObtenirOrigine() + I.ObtenirDistance() * Rayon.ObtenirDirection();
        CRayon LR;
        for (auto* L : Lumieres) {
            LR.AjusterOrigine(P);
            LR.AjusterDirection(L->GetPosition() - P);
            LR.AjusterEnergie(1);
            LR.AjusterIndiceRefraction(1);
            if (CVecteur3::ProdScal(LR.ObtenirDirection(), I.ObtenirNormale()) > 0) {
                CCouleur Filter = ObtenirFiltreDeSurface(LR);
                CCouleur LC = L->ObtenirCouleur() * Filter;
                REAL Gouraud = L->GetIntensity() * I.ObtenirSurface()->ObtenirCoeffDiffus() *
                               CVecteur3::ProdScal(I.ObtenirNormale(), LR.ObtenirDirection());
                Result += I.ObtenirSurface()->ObtenirCouleur() * Gouraud * LC;
                CVecteur3 Rf = CVecteur3::Reflect(LR.ObtenirDirection(), I.ObtenirNormale());
                REAL PS = CVecteur3::ProdScal(Rf, Rayon.ObtenirDirection());
                if (PS > 0) {
                    REAL Phong = L->GetIntensity() * I.ObtenirSurface()->ObtenirCoeffSpeculaire() *
                                 pow(PS, I.ObtenirSurface()->ObtenirCoeffBrillance());
                    Result += (Phong * LC);
                }
            }
        }
        REAL ReflE = I.ObtenirSurface()->ObtenirCoeffReflexion() * Rayon.ObtenirEnergie();
        if (ReflE > EnergieMinRayon && Rayon.ObtenirNbRebonds() < NbRebondsMax) {
            CRayon RR;
            RR.AjusterDirection(CVecteur3::Reflect(Rayon.ObtenirDirection(), I.ObtenirNormale()));
            RR.AjusterOrigine(P);
            RR.AjusterEnergie(ReflE);
            RR.AjusterNbRebonds(Rayon.ObtenirNbRebonds() + 1);
            Result += ObtenirCouleur(RR) * I.ObtenirSurface()->ObtenirCoeffReflexion();
        }
        REAL RefrE = I.ObtenirSurface()->ObtenirCoeffRefraction() * Rayon.ObtenirEnergie();
        if (RefrE > EnergieMinRayon && Rayon.ObtenirNbRebonds() < NbRebondsMax) {
            REAL Ratio;
            CRayon TR;
            CVecteur3 N = I.ObtenirNormale();
            if (Rayon.ObtenirIndiceRefraction() == I.ObtenirSurface()->ObtenirIndiceRefraction()) {
                TR.AjusterIndiceRefraction(IndiceRefractionScene);
                Ratio = I.ObtenirSurface()->ObtenirIndiceRefraction() / IndiceRefractionScene;
                N = -N;
            } else {
                TR.AjusterIndiceRefraction(I.ObtenirSurface()->ObtenirIndiceRefraction());
                Ratio = IndiceRefractionScene / I.ObtenirSurface()->ObtenirIndiceRefraction();
            }
            TR.AjusterOrigine(P);
            TR.AjusterEnergie(RefrE);
            TR.AjusterNbRebonds(Rayon.ObtenirNbRebonds() + 1);
            TR.AjusterDirection(CVecteur3::Refract(Rayon.ObtenirDirection(), N, Ratio));
            Result += ObtenirCouleur(TR) * I.ObtenirSurface()->ObtenirCoeffRefraction();
        }
        return Result;
    }

    // Scene.cpp:1842-1861
    CCouleur ObtenirFiltreDeSurface(CRayon& LR) const
    {
        CCouleur Filter = CCouleur::BLANC;
        CIntersection LI;
        REAL Distance = CVecteur3::Norme(LR.ObtenirDirection());
        LR.AjusterDirection(LR.ObtenirDirection() / Distance);
        for (auto* s : Surfaces) {
            LI = s->Intersection(LR);
            if (LI.ObtenirDistance() > EPSILON && LI.ObtenirDistance() < Distance)
                Filter *= LI.ObtenirSurface()->ObtenirCouleur() * LI.ObtenirSurface()->ObtenirCoeffRefraction();
        }
        return Filter;
    }

    // Scene.cpp:1538-1561 loop body
    CCouleur Pixel(int PixX, int PixY) const
    {
        CRayon Rayon;
        Rayon.AjusterOrigine(Camera.Position);
        Rayon.AjusterDirection(CVecteur3((2 * PixX * InvW - 1) * HalfW, (2 * PixY * InvH - 1) * HalfH, -1));
        Rayon.AjusterDirection(CVecteur3::Normaliser(Rayon.ObtenirDirection() * Camera.Orientation));
        Rayon.AjusterEnergie(1);
        Rayon.AjusterNbRebonds(0);
        Rayon.AjusterIndiceRefraction(1);
        return ObtenirCouleur(Rayon);
    }
};

}  // namespace

REXPORT int ref_load(const char* path, int w, int h, int max_bounces, void** out)
{
    RefScene* S = new RefScene();
    *out = S;
    S->ResLargeur = w;
    S->ResHauteur = h;
    S->NbRebondsMax = max_bounces;
    int rc = S->Traiter(path);
    if (rc) return rc;
    S->Initialiser();
    return 0;
}

// An explicit camera, as the product's rt_frame carries it (include/rt.h):
// position, the 4x4 orientation (row-major m[i][j]), the film half extents
// and the pixel reciprocals — the state Scene.cpp:1538-1561 reads per pixel
// (Camera.Position, Camera.Orientation, HalfW/HalfH from :676-677,
// InvW/InvH from :678-679).  What a caller that moves the camera between
// frames (Main.cpp:229-250, LancerRayons per frame) hands the pixel loop.
REXPORT int ref_set_camera(void* sp, const float* pos, const float* orient, float half_w, float half_h, float inv_w,
                           float inv_h, int w, int h)
{
    RefScene* S = (RefScene*)sp;
    S->Camera.Position = CVecteur3(pos[0], pos[1], pos[2]);
    S->Camera.Orientation = CMatrice4(orient[0], orient[1], orient[2], orient[3], orient[4], orient[5], orient[6],
                                      orient[7], orient[8], orient[9], orient[10], orient[11], orient[12],
                                      orient[13], orient[14], orient[15]);
    S->HalfW = half_w;
    S->HalfH = half_h;
    S->InvW = inv_w;
    S->InvH = inv_h;
    S->ResLargeur = w;
    S->ResHauteur = h;
    return 0;
}

REXPORT const char* ref_error(void* s) { return ((RefScene*)s)->err.c_str(); }
REXPORT void ref_free(void* s) { delete (RefScene*)s; }

REXPORT int ref_render_window(void* sp, int row0, int row1, int col0, int col1, float* rgb)
{
    RefScene* S = (RefScene*)sp;
    int ww = col1 - col0;
    for (int y = row0; y < row1; y++)
        for (int x = col0; x < col1; x++) {
            CCouleur c = S->Pixel(x, y);
            float* o = rgb + ((size_t)(y - row0) * ww + (x - col0)) * 3;
            o[0] = c.r;
            o[1] = c.g;
            o[2] = c.b;
        }
    return 0;
}

REXPORT int ref_counts(void* sp, int* nsurf, int* nlights)
{
    RefScene* S = (RefScene*)sp;
    *nsurf = (int)S->Surfaces.size();
    *nlights = (int)S->Lumieres.size();
    return 0;
}

// Same canonical layout as oracle_dump (rt_oracle.c).
REXPORT int ref_dump(void* sp, float* surf, float* cam, float* lights)
{
    RefScene* S = (RefScene*)sp;
    for (size_t i = 0; i < S->Surfaces.size(); i++) {
        ISurface* s = S->Surfaces[i];
        float* o = surf + i * 24;
        memset(o, 0, 24 * sizeof(float));
        o[0] = (float)S->Types[i];
        CCouleur c = s->ObtenirCouleur();
        o[1] = c.r; o[2] = c.g; o[3] = c.b;
        o[4] = s->ObtenirCoeffAmbiant(); o[5] = s->ObtenirCoeffDiffus();
        o[6] = s->ObtenirCoeffSpeculaire(); o[7] = s->ObtenirCoeffBrillance();
        o[8] = s->ObtenirCoeffReflexion(); o[9] = s->ObtenirCoeffRefraction();
        o[10] = s->ObtenirIndiceRefraction();
        if (S->Types[i] == 0) {
            CTriangle* t = (CTriangle*)s;
            for (int k = 0; k < 3; k++) {
                CVecteur3 p = t->ObtenirPoint(k);
                o[11 + 3 * k] = p.x; o[12 + 3 * k] = p.y; o[13 + 3 * k] = p.z;
            }
            CVecteur3 n = t->ObtenirNormale();
            o[20] = n.x; o[21] = n.y; o[22] = n.z;
        } else if (S->Types[i] == 1) {
            CPlan* p = (CPlan*)s;
            CVecteur3 n = p->ObtenirNormale();
            o[11] = n.x; o[12] = n.y; o[13] = n.z; o[14] = p->ObtenirConstante();
        } else {
            CQuadrique* q = (CQuadrique*)s;
            CVecteur3 a = q->ObtenirQuadratique(), l = q->ObtenirLineaire(), m = q->ObtenirMixte();
            o[11] = a.x; o[12] = a.y; o[13] = a.z;
            o[14] = l.x; o[15] = l.y; o[16] = l.z;
            o[17] = m.x; o[18] = m.y; o[19] = m.z;
            o[20] = q->ObtenirConstante();
        }
    }
    cam[0] = S->Camera.Position.x; cam[1] = S->Camera.Position.y; cam[2] = S->Camera.Position.z;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) cam[3 + 4 * i + j] = S->Camera.Orientation.m[i][j];
    cam[19] = S->Camera.Angle; cam[20] = S->HalfW; cam[21] = S->HalfH;
    cam[22] = S->InvW; cam[23] = S->InvH;
    cam[24] = S->CouleurArrierePlan.r; cam[25] = S->CouleurArrierePlan.g; cam[26] = S->CouleurArrierePlan.b;
    for (size_t i = 0; i < S->Lumieres.size(); i++) {
        CLumiere* L = S->Lumieres[i];
        float* o = lights + i * 7;
        CVecteur3 p = L->GetPosition();
        CCouleur c = L->ObtenirCouleur();
        o[0] = p.x; o[1] = p.y; o[2] = p.z;
        o[3] = c.r; o[4] = c.g; o[5] = c.b;
        o[6] = L->GetIntensity();
    }
    return 0;
}

// Per-primitive known answers through the reference's own Intersection():
// geometry words as in oracle_intersect (post-Pretraitement values, identity
// transform so Pretraitement is not re-applied).
REXPORT int ref_intersect(int type, const float* g, const float* ro, const float* rd, float* t_out, float* n_out)
{
    CRayon R;
    R.AjusterOrigine(CVecteur3(ro[0], ro[1], ro[2]));
    R.AjusterDirection(CVecteur3(rd[0], rd[1], rd[2]));
    R.AjusterEnergie(1);
    R.AjusterIndiceRefraction(1);
    CIntersection I;
    if (type == 0) {
        CTriangle t;
        t.AjusterPoints(CVecteur3(g[0], g[1], g[2]), CVecteur3(g[3], g[4], g[5]), CVecteur3(g[6], g[7], g[8]));
        t.AjusterNormale(CVecteur3(g[9], g[10], g[11]));
        I = t.Intersection(R);
    } else if (type == 1) {
        CPlan p;
        p.AjusterNormale(CVecteur3(g[0], g[1], g[2]));
        p.AjusterConstante(g[3]);
        I = p.Intersection(R);
    } else {
        CQuadrique q;
        q.AjusterQuadratique(CVecteur3(g[0], g[1], g[2]));
        q.AjusterLineaire(CVecteur3(g[3], g[4], g[5]));
        q.AjusterMixte(CVecteur3(g[6], g[7], g[8]));
        q.AjusterConstante(g[9]);
        I = q.Intersection(R);
    }
    *t_out = I.ObtenirDistance();
    CVecteur3 n = I.ObtenirNormale();
    n_out[0] = n.x; n_out[1] = n.y; n_out[2] = n.z;
    return I.ObtenirSurface() != nullptr;
}
