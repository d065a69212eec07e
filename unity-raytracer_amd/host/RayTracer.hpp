// RayTracer.hpp — C++ host mirror of the reference's render interface, on
// top of the C-ABI (include/rt_mi355.h).
//
// The reference is C#/Unity (vectorized-runner/unity-raytracer @ v1); its
// toolchain is absent here, so the host side above the boundary is C++ with
// the reference's names and meanings:
//   RayTracer::Scene            Data/Objects/Scene.cs:6-15 (TriangleData, MeshData,
//                               SphereData, PointLights, AmbientLight; CalculateAABB)
//   RayTracer::Mesh             Data/Objects/Mesh.cs:7-13
//   RayTracer::MaterialData     Data/Shading/MaterialData.cs:7-15
//   RayTracer::CameraData       Data/Camera/CameraData.cs:5-11
//   RayTracer::ImagePlane       Data/Camera/ImagePlane.cs:11-45
//   RayTracer::RayTracingSetup  Demo-RayTracing/RayTracingSetup.cs: fields ImagePlane,
//                               BackgroundColor, MaxReflectionBounces, Scene, PixelColors;
//                               CastPixelRays(CameraData) :275-302
//   RayTracer::Triangle::Normal Data/Objects/Triangle.cs:13-21
// Errors: the reference logs (Debug.LogError) or throws; here a failing
// C-ABI call throws RayTracer::Error carrying rt_status and rt_last_error().
#pragma once

#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt_mi355.h"

namespace RayTracer {

using float3 = rt_float3;

inline float3 operator+(float3 a, float3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float3 operator-(float3 a, float3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }

struct Color {  // UnityEngine.Color
    float r = 0, g = 0, b = 0, a = 1;
};

struct Triangle {
    float3 Vertex0{}, Vertex1{}, Vertex2{};
    // Triangle.Normal: v / length(v), v = cross(Vertex2 - Vertex0, Vertex1 - Vertex0)
    float3 Normal() const {
        const float3 a = Vertex2 - Vertex0, b = Vertex1 - Vertex0;
        const float3 v{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
        const float len = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
        return {v.x / len, v.y / len, v.z / len};
    }
};

struct Sphere {
    float3 Center{};
    float RadiusSquared = 0;
};

struct AABB {
    float3 Min{}, Max{};
};

struct MaterialData {
    float3 DiffuseReflectance{}, AmbientReflectance{}, MirrorReflectance{}, SpecularReflectance{};
    float PhongExponent = 0;
    bool IsMirror = false;
    rt_material abi() const {
        return rt_material{DiffuseReflectance, AmbientReflectance, MirrorReflectance, SpecularReflectance,
                           PhongExponent, IsMirror ? 1 : 0};
    }
};

struct Mesh {
    std::vector<Triangle> Triangles;
    std::vector<float3> TriangleNormals;  // -Triangle.Normal (SceneMesh.cs:43)
    MaterialData Material;
    AABB Bounds;
};

struct TriangleData {
    std::vector<Triangle> Triangles;
    std::vector<float3> Normals;
    std::vector<MaterialData> Materials;
};

struct MeshData {
    std::vector<Mesh> Meshes;
};

struct SphereData {
    std::vector<Sphere> Spheres;
    std::vector<MaterialData> Materials;
};

struct PointLightData {
    float3 Position{}, Intensity{};
};

struct AmbientLightData {
    float3 Radiance{};
};

struct Scene {
    TriangleData Triangles;
    MeshData Meshes;
    SphereData Spheres;
    std::vector<PointLightData> PointLights;
    AmbientLightData AmbientLight;
};

struct CameraData {
    float3 Position{0, 0, 0}, Forward{0, 0, 1}, Right{1, 0, 0}, Up{0, 1, 0};
};

struct ImagePlane {
    int ResolutionX = 0, ResolutionY = 0;
    float DistanceToCamera = 0, HalfHorizontalLength = 0, HalfVerticalLength = 0;
};

class Error : public std::runtime_error {
   public:
    Error(int status, const std::string &msg) : std::runtime_error(msg), status(status) {}
    int status;
};

class RayTracingSetup {
   public:
    ImagePlane ImagePlane_;
    Color BackgroundColor;
    int MaxReflectionBounces = 0;
    int SamplesPerPixel = 1;  // n*n extension; 1 == reference
    Scene Scene_;
    std::vector<Color> PixelColors;
    rt_stats LastStats{};

    RayTracingSetup() {
        int st = rt_create(&ctx_, 1);
        if (st != RT_OK) throw Error(st, rt_last_error(nullptr));
    }
    ~RayTracingSetup() { rt_destroy(ctx_); }
    RayTracingSetup(const RayTracingSetup &) = delete;
    RayTracingSetup &operator=(const RayTracingSetup &) = delete;

    // UpdateScene() result upload (:120-128): flattens the lists and hands
    // them to rt_set_scene (which computes Scene.CalculateAABB + the BVH).
    void UpdateScene() {
        std::vector<rt_triangle> tris, mesh_tris;
        std::vector<rt_material> tri_mats, sph_mats;
        std::vector<rt_float3> mesh_normals;
        std::vector<rt_mesh> meshes;
        std::vector<rt_sphere> spheres;
        std::vector<rt_point_light> lights;
        for (const Triangle &t : Scene_.Triangles.Triangles) tris.push_back({t.Vertex0, t.Vertex1, t.Vertex2});
        for (const MaterialData &m : Scene_.Triangles.Materials) tri_mats.push_back(m.abi());
        for (const Mesh &m : Scene_.Meshes.Meshes) {
            rt_mesh d{};
            d.first_triangle = (int32_t)mesh_tris.size();
            d.triangle_count = (int32_t)m.Triangles.size();
            d.material = m.Material.abi();
            d.aabb = {m.Bounds.Min, m.Bounds.Max};
            for (const Triangle &t : m.Triangles) mesh_tris.push_back({t.Vertex0, t.Vertex1, t.Vertex2});
            mesh_normals.insert(mesh_normals.end(), m.TriangleNormals.begin(), m.TriangleNormals.end());
            meshes.push_back(d);
        }
        for (const Sphere &s : Scene_.Spheres.Spheres) spheres.push_back({s.Center, s.RadiusSquared});
        for (const MaterialData &m : Scene_.Spheres.Materials) sph_mats.push_back(m.abi());
        for (const PointLightData &l : Scene_.PointLights) lights.push_back({l.Position, l.Intensity});
        rt_scene_desc d{};
        d.triangles = tris.data();
        d.triangle_normals = Scene_.Triangles.Normals.data();
        d.triangle_materials = tri_mats.data();
        d.triangle_count = (int32_t)tris.size();
        d.mesh_triangles = mesh_tris.data();
        d.mesh_triangle_normals = mesh_normals.data();
        d.mesh_triangle_total = (int32_t)mesh_tris.size();
        d.meshes = meshes.data();
        d.mesh_count = (int32_t)meshes.size();
        d.spheres = spheres.data();
        d.sphere_materials = sph_mats.data();
        d.sphere_count = (int32_t)spheres.size();
        d.point_lights = lights.data();
        d.point_light_count = (int32_t)lights.size();
        d.ambient_radiance = Scene_.AmbientLight.Radiance;
        check(rt_set_scene(ctx_, &d));
    }

    // CastPixelRays(CameraData), RayTracingSetup.cs:275-302
    void CastPixelRays(const CameraData &cam) {
        const rt_camera c{cam.Position, cam.Forward, cam.Right, cam.Up};
        const rt_image_plane p{ImagePlane_.ResolutionX, ImagePlane_.ResolutionY, ImagePlane_.DistanceToCamera,
                               ImagePlane_.HalfHorizontalLength, ImagePlane_.HalfVerticalLength};
        rt_render_params prm{};
        prm.background_color[0] = BackgroundColor.r;
        prm.background_color[1] = BackgroundColor.g;
        prm.background_color[2] = BackgroundColor.b;
        prm.background_color[3] = BackgroundColor.a;
        prm.max_reflection_bounces = MaxReflectionBounces;
        prm.samples_per_pixel = SamplesPerPixel;
        prm.band_count = 1;
        PixelColors.assign((size_t)std::max(0, ImagePlane_.ResolutionX) * std::max(0, ImagePlane_.ResolutionY),
                           Color{});
        check(rt_render(ctx_, &c, &p, &prm, reinterpret_cast<float *>(PixelColors.data()), &LastStats));
    }

    rt_ctx *context() const { return ctx_; }

   private:
    void check(int st) {
        if (st != RT_OK) throw Error(st, rt_last_error(ctx_));
    }
    rt_ctx *ctx_ = nullptr;
};

static_assert(sizeof(Color) == 16, "Color is RGBA float32 like UnityEngine.Color");

}  // namespace RayTracer
