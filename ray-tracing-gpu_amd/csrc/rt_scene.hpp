// rt_scene.hpp — host-side mirror of the reference's CScene surface
// (Scene.h:30-179): scene-file loader, camera, Pretraitement, and the
// flattening of m_Surfaces / m_Lumieres (FILE ORDER) into the rt_scene_flat
// arrays the device consumes.  No GL, no singleton, no exits.
#pragma once

#include <string>
#include <vector>

#include "../../include/rt.h"
#include "rt_math.h"

namespace rt {

enum class SurfaceKind : int { Triangle = RT_TRIANGLE, Plane = RT_PLANE, Quadric = RT_QUADRIC };

// ISurface.h:25-41 with the defaults of ISurface.cpp:15-25.
struct Material {
    Color color{0.f, 0.f, 0.f};  // CCouleur::NOIR
    float ka = 0.2f, kd = 0.8f, ks = 0.0f, shininess = 0.0f;
    float kr = 0.0f, kt = 0.0f, ior = 0.0f;
};

struct Surface {
    SurfaceKind kind;
    Material mat;
    Mat4 xform = identity4();
    Vec3 pts[3]{};     // triangle: m_Pts
    Vec3 normal{};     // triangle / plane: m_Normale
    Vec3 quad{}, lin{}, mix{};  // quadric
    float cst = 0.0f;  // plane / quadric: m_Cst

    void Pretraitement();
};

// Lumiere.h:23-27 / Lumiere.cpp defaults (white, intensity 0).
struct Light {
    Vec3 pos{0.f, 0.f, 0.f};
    Color color{1.f, 1.f, 1.f};
    float intensity = 0.0f;
};

class Scene {
public:
    // Scene.cpp:61-88 constructor defaults.
    int width = 0, height = 0;
    int max_bounces = 20;       // m_NbRebondsMax
    float min_energy = 0.01f;   // m_EnergieMinRayon
    float scene_ior = 1.0f;     // m_IndiceRefractionScene
    Color background{0.f, 0.f, 0.f};
    Vec3 cam_pos{0.f, 0.f, 0.f}, cam_eye{0.f, 0.f, 0.f}, cam_up{0.f, 1.f, 0.f};
    float focale = 50.0f, angle = 0.0f;
    Mat4 orientation = identity4();
    float half_w = 0.f, half_h = 0.f, inv_w = 0.f, inv_h = 0.f;

    std::vector<Surface> surfaces;
    std::vector<Light> lights;
    bool loaded = false, prepared = false;
    std::string error;

    int TraiterFichierDeScene(const char* path);
    int Initialiser();  // camera + Pretraitement + LancerRayons prologue
    void InitialiserCamera();

    // Flat views handed across the C ABI (valid until the next prepare).
    std::vector<int32_t> flat_type;
    std::vector<float> flat_geom, flat_mat, flat_lights;
    void Flatten();
};

}  // namespace rt
