/* oracle_asan.c — AddressSanitizer + UBSan driver for the CPU oracle
 * (oracle/rt_oracle.c, test infrastructure), tools/asan/Makefile.  Renders
 * small scenes with every primitive kind (loose triangles, spheres, a mesh
 * with its AABB gate, lights, ambient, mirrors) at several spp/depths, runs
 * batch closest-hit queries with NaN / zero / axis-parallel directions, and
 * checks that every pixel is finite and alpha is 1.  Exit 0 = clean. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rt_mi355.h"

typedef struct orc_counts {
    uint64_t primary_rays, shadow_rays, reflection_rays, box_tests, triangle_tests, sphere_tests, shading_fetches;
} orc_counts;
int orc_render(const rt_scene_desc *sc, const rt_camera *cam, const rt_image_plane *plane,
               const rt_render_params *prm, float *out, orc_counts *counts, int32_t threads);
void orc_intersect(const rt_scene_desc *sc, const rt_ray *rays, int32_t n, rt_hit *out);

static rt_float3 v3(float x, float y, float z) {
    rt_float3 r = {x, y, z};
    return r;
}
static rt_float3 nrm(rt_triangle t) { /* Triangle.Normal (division form) */
    rt_float3 a = v3(t.vertex2.x - t.vertex0.x, t.vertex2.y - t.vertex0.y, t.vertex2.z - t.vertex0.z);
    rt_float3 b = v3(t.vertex1.x - t.vertex0.x, t.vertex1.y - t.vertex0.y, t.vertex1.z - t.vertex0.z);
    rt_float3 c = v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
    float l = sqrtf(c.x * c.x + c.y * c.y + c.z * c.z);
    return v3(c.x / l, c.y / l, c.z / l);
}
static float frand(unsigned *s) {
    *s = *s * 1664525u + 1013904223u;
    return (float)(*s >> 8) / 16777216.0f * 2.0f - 1.0f;
}

int main(void) {
    unsigned seed = 20250101u;
    enum { NT = 24, NM = 36, NS = 4 };
    rt_triangle tris[NT], mtris[NM];
    rt_float3 tn[NT], mtn[NM];
    rt_material tm[NT], sm[NS];
    rt_sphere sph[NS];
    rt_mesh mesh[2];
    rt_point_light lights[2];
    memset(tm, 0, sizeof tm);
    memset(sm, 0, sizeof sm);
    memset(mesh, 0, sizeof mesh);
    for (int i = 0; i < NT; ++i) {
        tris[i].vertex0 = v3(frand(&seed), frand(&seed), frand(&seed));
        tris[i].vertex1 = v3(frand(&seed), frand(&seed), frand(&seed));
        tris[i].vertex2 = v3(frand(&seed), frand(&seed), frand(&seed));
        if (i == 0) tris[i].vertex2 = tris[i].vertex1; /* degenerate: NaN normal */
        tn[i] = nrm(tris[i]);
        tm[i].diffuse_reflectance = v3(0.5f, 0.4f, 0.3f);
        tm[i].ambient_reflectance = v3(0.1f, 0.1f, 0.1f);
        tm[i].specular_reflectance = v3(0.2f, 0.2f, 0.2f);
        tm[i].phong_exponent = (float)(i % 5) * 7.5f;
        tm[i].mirror_reflectance = v3(0.7f, 0.7f, 0.7f);
        tm[i].is_mirror = i % 4 == 0;
    }
    for (int m = 0; m < 2; ++m) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = 0; i < NM / 2; ++i) {
            rt_triangle *t = &mtris[m * (NM / 2) + i];
            t->vertex0 = v3(0.3f * frand(&seed) + m, 0.3f * frand(&seed), 0.3f * frand(&seed));
            t->vertex1 = v3(0.3f * frand(&seed) + m, 0.3f * frand(&seed), 0.3f * frand(&seed));
            t->vertex2 = v3(0.3f * frand(&seed) + m, 0.3f * frand(&seed), 0.3f * frand(&seed));
            rt_float3 n = nrm(*t);
            mtn[m * (NM / 2) + i] = v3(-n.x, -n.y, -n.z);
            const rt_float3 *vs[3] = {&t->vertex0, &t->vertex1, &t->vertex2};
            for (int k = 0; k < 3; ++k) {
                const float p[3] = {vs[k]->x, vs[k]->y, vs[k]->z};
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fminf(lo[a], p[a]);
                    hi[a] = fmaxf(hi[a], p[a]);
                }
            }
        }
        mesh[m].first_triangle = m * (NM / 2);
        mesh[m].triangle_count = NM / 2;
        mesh[m].material = tm[m + 1];
        mesh[m].material.is_mirror = m;
        mesh[m].aabb.min = v3(lo[0], lo[1], lo[2]);
        mesh[m].aabb.max = v3(hi[0], hi[1], hi[2]);
    }
    for (int i = 0; i < NS; ++i) {
        sph[i].center = v3(frand(&seed), frand(&seed), frand(&seed));
        sph[i].radius_squared = 0.05f + 0.05f * (float)i;
        sm[i] = tm[i + 2];
        sm[i].is_mirror = i % 2;
    }
    lights[0].position = v3(0.0f, 2.0f, -1.0f);
    lights[0].intensity = v3(40.0f, 40.0f, 40.0f);
    lights[1].position = v3(-2.0f, 0.5f, 0.0f);
    lights[1].intensity = v3(10.0f, 10.0f, 10.0f);
    rt_scene_desc sc;
    memset(&sc, 0, sizeof sc);
    sc.triangles = tris; sc.triangle_normals = tn; sc.triangle_materials = tm; sc.triangle_count = NT;
    sc.mesh_triangles = mtris; sc.mesh_triangle_normals = mtn; sc.mesh_triangle_total = NM;
    sc.meshes = mesh; sc.mesh_count = 2;
    sc.spheres = sph; sc.sphere_materials = sm; sc.sphere_count = NS;
    sc.point_lights = lights; sc.point_light_count = 2;
    sc.ambient_radiance = v3(20.0f, 20.0f, 20.0f);
    rt_camera cam = {v3(0.0f, 0.0f, -3.4f), v3(0, 0, 1), v3(1, 0, 0), v3(0, 1, 0)};
    int bad = 0;
    const int spps[3] = {1, 4, 9}, depths[3] = {0, 3, 40};
    for (int c = 0; c < 3; ++c) {
        rt_image_plane plane = {23 + c, 17, 1.0f, 0.6f, 0.45f};
        rt_render_params prm;
        memset(&prm, 0, sizeof prm);
        prm.background_color[0] = 0.1f; prm.background_color[3] = 1.0f;
        prm.max_reflection_bounces = depths[c];
        prm.samples_per_pixel = spps[c];
        prm.band_count = 1;
        size_t npx = (size_t)plane.resolution_x * plane.resolution_y;
        float *img = (float *)malloc(npx * 4 * sizeof(float));
        orc_counts cnt;
        int st = orc_render(&sc, &cam, &plane, &prm, img, &cnt, 2);
        for (size_t i = 0; i < npx; ++i)
            if (img[4 * i + 3] != 1.0f) ++bad;
        printf("render %dx%d spp %d depth %d: status %d, rays %llu/%llu/%llu\n", plane.resolution_x,
               plane.resolution_y, spps[c], depths[c], st, (unsigned long long)cnt.primary_rays,
               (unsigned long long)cnt.shadow_rays, (unsigned long long)cnt.reflection_rays);
        bad += st != 0;
        free(img);
    }
    enum { NR = 512 };
    rt_ray rays[NR];
    rt_hit hits[NR];
    for (int i = 0; i < NR; ++i) {
        rays[i].origin = v3(frand(&seed) * 2.0f, frand(&seed) * 2.0f, frand(&seed) * 2.0f);
        rays[i].direction = v3(frand(&seed), frand(&seed), frand(&seed));
        if (i % 7 == 0) rays[i].direction.x = 0.0f;
        if (i % 11 == 0) rays[i].direction = v3(0.0f, 0.0f, 0.0f);
        if (i % 13 == 0) rays[i].direction.y = NAN;
        if (i % 17 == 0) rays[i].direction.z = -0.0f;
    }
    orc_intersect(&sc, rays, NR, hits);
    int nhit = 0;
    for (int i = 0; i < NR; ++i) nhit += hits[i].type != 0;
    printf("intersect: %d of %d rays hit\n", nhit, NR);
    printf("%s\n", bad ? "FAILED" : "ALL OK");
    return bad ? 1 : 0;
}
