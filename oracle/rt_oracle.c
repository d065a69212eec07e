/*
 * rt_oracle.c — CPU ORACLE (test infrastructure, NOT the product).
 *
 * A plain-C, single-precision restatement of the reference's per-pixel trace
 * loop (vectorized-runner/unity-raytracer @ v1, C#/Unity, not buildable here:
 * no dotnet/mono/Unity in this image — see DESIGN.md "Oracle").  It follows
 * the reference operation for operation, including its brute-force
 * closest-hit scan and the literal recursion of Shade().  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math, SSE
 * float32 so every + - * / sqrt is one IEEE-754 single rounding).
 *
 * Parity pinning: the reference ships one known answer
 * (Assets/RayTracer/Tests/RayTracerTests.cs:11-26: t = 299) and no golden
 * images.  Unity.Mathematics 1.2.6 (not vendored) is restated from its
 * public source; that boundary is "parity unpinned" (DESIGN.md).  The
 * restatement is cross-checked bit for bit against an independent numpy
 * float32 restatement (oracle/np_oracle.py) on the committed fixtures.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#include "../include/rt_mi355.h"

/* ------------------------------------------------------------------------
 * Unity.Mathematics 1.2.6 restated (package source, math.cs / float3.gen.cs)
 * --------------------------------------------------------------------- */
typedef rt_float3 f3;

static inline f3 V(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add(f3 a, f3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub(f3 a, f3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul(f3 a, f3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 muls(f3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }       /* float3 * float */
static inline f3 smul(float s, f3 a) { return V(s * a.x, s * a.y, s * a.z); }       /* float * float3 */
static inline f3 divs(f3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }       /* float3 / float */
static inline f3 neg(f3 a) { return V(-a.x, -a.y, -a.z); }
/* dot(x, y) = x.x*y.x + x.y*y.y + x.z*y.z, left to right */
static inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* cross(x, y) = (x * y.yzx - x.yzx * y).yzx */
static inline f3 cross(f3 x, f3 y) {
    return V(x.y * y.z - x.z * y.y, x.z * y.x - x.x * y.z, x.x * y.y - x.y * y.x);
}
static inline float lengthsq(f3 a) { return dot(a, a); }
/* sqrt(float) = (float)System.Math.Sqrt(x): double sqrt of a float rounded
 * to float equals the correctly rounded float sqrt. */
static inline float length(f3 a) { return sqrtf(dot(a, a)); }
/* rsqrt(x) = 1.0f / sqrt(x);  normalize(x) = rsqrt(dot(x, x)) * x */
static inline f3 normalize(f3 a) { float r = 1.0f / sqrtf(dot(a, a)); return smul(r, a); }
/* distancesq(x, y) = lengthsq(y - x) */
static inline float distancesq(f3 x, f3 y) { return lengthsq(sub(y, x)); }
/* min(x, y) = isnan(y) || x < y ? x : y;  max(x, y) = isnan(y) || x > y ? x : y */
static inline float umin(float x, float y) { return (isnan(y) || x < y) ? x : y; }
static inline float umax(float x, float y) { return (isnan(y) || x > y) ? x : y; }
static inline f3 umin3(f3 a, f3 b) { return V(umin(a.x, b.x), umin(a.y, b.y), umin(a.z, b.z)); }
static inline f3 umax3(f3 a, f3 b) { return V(umax(a.x, b.x), umax(a.y, b.y), umax(a.z, b.z)); }
static inline float comp(f3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
/* acos/pow(float) = (float)System.Math.Acos/Pow((double)x ...) */
static inline float uacos(float x) { return (float)acos((double)x); }
static inline float upow(float x, float y) { return (float)pow((double)x, (double)y); }
/* degrees(x) = x * TODEGREES, TODEGREES = 57.29578f */
static inline float degrees(float x) { return x * 57.29578f; }

/* ------------------------------------------------------------------------
 * RMath, Assets/RayTracer/Math/RMath.cs
 * --------------------------------------------------------------------- */
#define RMATH_EPSILON 0.00001f /* RMath.cs:9 */

/* RMath.RayAABBIntersection, RMath.cs:12-26 */
int orc_ray_aabb(const rt_ray *ray, const rt_aabb *box) {
    f3 inv = V(1.0f / ray->direction.x, 1.0f / ray->direction.y, 1.0f / ray->direction.z); /* rcp */
    float tmin = 0.0f, tmax = INFINITY;
    for (int i = 0; i < 3; ++i) {
        float t1 = (comp(box->min, i) - comp(ray->origin, i)) * comp(inv, i);
        float t2 = (comp(box->max, i) - comp(ray->origin, i)) * comp(inv, i);
        tmin = umin(umax(t1, tmin), umax(t2, tmin));
        tmax = umax(umin(t1, tmax), umin(t2, tmax));
    }
    return tmin <= tmax;
}

/* RMath.RayTriangleIntersection (Möller–Trumbore, two-sided), RMath.cs:29-73 */
int orc_ray_triangle(const rt_ray *ray, const rt_triangle *tri, float *out_t) {
    f3 edge1 = sub(tri->vertex1, tri->vertex0);
    f3 edge2 = sub(tri->vertex2, tri->vertex0);
    f3 h = cross(ray->direction, edge2);
    float a = dot(edge1, h);
    *out_t = 0.0f;
    if (a > -RMATH_EPSILON && a < RMATH_EPSILON) return 0; /* parallel */
    float f = 1.0f / a;
    f3 s = sub(ray->origin, tri->vertex0);
    float u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return 0;
    f3 q = cross(s, edge1);
    float v = f * dot(ray->direction, q);
    if (v < 0.0f || u + v > 1.0f) return 0;
    float t = f * dot(edge2, q);
    if (t > RMATH_EPSILON) { *out_t = t; return 1; }
    return 0;
}

/* RMath.RaySphereIntersection, RMath.cs:81-108 (assumes a unit direction) */
int orc_ray_sphere(const rt_ray *ray, const rt_sphere *sph, float *out_t) {
    f3 oc = sub(ray->origin, sph->center);
    float uoc = dot(ray->direction, oc);
    float disc = uoc * uoc - (lengthsq(oc) - sph->radius_squared);
    *out_t = 0.0f;
    if (disc < 0) return 0;
    float sq = sqrtf(disc);
    float big = -uoc + sq;
    if (big < 0) return 0;
    float small = -uoc - sq;
    *out_t = small < 0 ? big : small;
    return 1;
}

/* Triangle.Normal, Data/Objects/Triangle.cs:13-21: v / length(v),
 * v = cross(Vertex2 - Vertex0, Vertex1 - Vertex0) (float3 / float division) */
void orc_triangle_normal(const rt_triangle *tri, rt_float3 *out) {
    f3 v = cross(sub(tri->vertex2, tri->vertex0), sub(tri->vertex1, tri->vertex0));
    *out = divs(v, length(v));
}

/* AABB.Encapsulate(float3), AABB.cs:10-14 */
static inline void encap_point(rt_aabb *b, f3 p) { b->min = umin3(p, b->min); b->max = umax3(p, b->max); }
/* AABB.Encapsulate(AABB), AABB.cs:16-20 */
static inline void encap_box(rt_aabb *b, rt_aabb o) { b->min = umin3(b->min, o.min); b->max = umax3(b->max, o.max); }

/* Scene.CalculateAABB, Data/Objects/Scene.cs:17-41.  float.MinValue is -FLT_MAX. */
void orc_scene_aabb(const rt_scene_desc *sc, rt_aabb *out) {
    rt_aabb b;
    b.min = V(FLT_MAX, FLT_MAX, FLT_MAX);
    b.max = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int m = 0; m < sc->mesh_count; ++m) encap_box(&b, sc->meshes[m].aabb);
    for (int i = 0; i < sc->triangle_count; ++i) {
        encap_point(&b, sc->triangles[i].vertex0);
        encap_point(&b, sc->triangles[i].vertex1);
        encap_point(&b, sc->triangles[i].vertex2);
    }
    for (int i = 0; i < sc->sphere_count; ++i) {
        /* Sphere.AABB, Sphere.cs:17-22: Center -/+ sqrt(RadiusSquared) */
        rt_sphere s = sc->spheres[i];
        float r = sqrtf(s.radius_squared);
        rt_aabb sb;
        sb.min = V(s.center.x - r, s.center.y - r, s.center.z - r);
        sb.max = V(s.center.x + r, s.center.y + r, s.center.z + r);
        encap_box(&b, sb);
    }
    *out = b;
}

/* Scene.IntersectRay, Data/Objects/Scene.cs:43-122 (brute force; strict '>'
 * so the first of equal distances wins). */
typedef struct { uint64_t box, tri, sph; } orc_tests;

static rt_hit intersect(const rt_scene_desc *sc, const rt_aabb *scene_box, const rt_ray *ray,
                        orc_tests *ct) {
    rt_hit hit;
    hit.type = 0; hit.index = -1; hit.mesh_index = -1;
    float best = FLT_MAX; /* float.MaxValue */
    ct->box++;
    if (!orc_ray_aabb(ray, scene_box)) { hit.distance = best; return hit; }
    for (int m = 0; m < sc->mesh_count; ++m) {
        const rt_mesh *mesh = &sc->meshes[m];
        ct->box++;
        if (!orc_ray_aabb(ray, &mesh->aabb)) continue;
        for (int i = 0; i < mesh->triangle_count; ++i) {
            float t;
            ct->tri++;
            if (orc_ray_triangle(ray, &sc->mesh_triangles[mesh->first_triangle + i], &t)) {
                if (best > t) { best = t; hit.type = 3; hit.index = i; hit.mesh_index = m; }
            }
        }
    }
    for (int i = 0; i < sc->sphere_count; ++i) {
        float t;
        ct->sph++;
        if (orc_ray_sphere(ray, &sc->spheres[i], &t)) {
            if (best > t) { best = t; hit.type = 1; hit.index = i; }
        }
    }
    for (int i = 0; i < sc->triangle_count; ++i) {
        float t;
        ct->tri++;
        if (orc_ray_triangle(ray, &sc->triangles[i], &t)) {
            if (best > t) { best = t; hit.type = 2; hit.index = i; }
        }
    }
    hit.distance = best;
    return hit;
}

void orc_intersect(const rt_scene_desc *sc, const rt_ray *rays, int32_t n, rt_hit *out) {
    rt_aabb box;
    orc_scene_aabb(sc, &box);
    orc_tests ct = {0, 0, 0};
    for (int32_t i = 0; i < n; ++i) out[i] = intersect(sc, &box, &rays[i], &ct);
}

/* ------------------------------------------------------------------------
 * RayTracingSetup render part, Assets/RayTracer/Demo-RayTracing/RayTracingSetup.cs
 * --------------------------------------------------------------------- */
#define SHADOW_RAY_EPSILON 0.0001f /* RayTracingSetup.cs:42 */

typedef struct orc_counts {
    uint64_t primary_rays, shadow_rays, reflection_rays;
    uint64_t box_tests, triangle_tests, sphere_tests, shading_fetches;
} orc_counts;

/* ------------------------------------------------------------------------
 * Optional CPU BVH for the closest-hit query (CPU-baseline only: separates
 * the algorithmic speed-up of a BVH from the GPU's).  Same answer as the
 * brute-force scan: the exact scene and per-mesh AABB gates, padded node
 * boxes that never cull a primitive the exact tests accept, ties to the
 * lowest reference rank (meshes, then spheres, then loose triangles, each in
 * order) — which is the scan's strict-'>' first-wins rule.
 * --------------------------------------------------------------------- */
typedef struct {
    float lo[3], hi[3];
    int first, count; /* count > 0: leaf over prim[first .. first+count); else children first, first+1 */
} bnode;

typedef struct orc_bvh {
    int n, nnodes, mesh_count, mt, ns;
    int *prim;        /* ranks in leaf order */
    int *mesh_of;     /* rank -> mesh (mesh triangles) */
    float *plo, *phi; /* padded bounds per rank */
    bnode *nodes;
} orc_bvh;

static const float *g_sort_c;  /* build-time comparator state (single-threaded build) */
static int g_sort_axis;
static int cmp_centroid(const void *a, const void *b) {
    const float ca = g_sort_c[3 * *(const int *)a + g_sort_axis], cb = g_sort_c[3 * *(const int *)b + g_sort_axis];
    if (ca < cb) return -1;
    if (ca > cb) return 1;
    return *(const int *)a - *(const int *)b;
}

static int bvh_build_rec(orc_bvh *B, const float *cen, int first, int count, int node) {
    bnode *nd = &B->nodes[node];
    for (int a = 0; a < 3; ++a) { nd->lo[a] = INFINITY; nd->hi[a] = -INFINITY; }
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = first; i < first + count; ++i) {
        const int r = B->prim[i];
        for (int a = 0; a < 3; ++a) {
            nd->lo[a] = fminf(nd->lo[a], B->plo[3 * r + a]);
            nd->hi[a] = fmaxf(nd->hi[a], B->phi[3 * r + a]);
            clo[a] = fminf(clo[a], cen[3 * r + a]);
            chi[a] = fmaxf(chi[a], cen[3 * r + a]);
        }
    }
    if (count <= 4) {
        nd->first = first;
        nd->count = count;
        return node + 1;
    }
    int axis = 0;
    for (int a = 1; a < 3; ++a)
        if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
    g_sort_c = cen;
    g_sort_axis = axis;
    qsort(B->prim + first, (size_t)count, sizeof(int), cmp_centroid);
    const int half = count / 2, left = node + 1;
    const int right = bvh_build_rec(B, cen, first, half, left);
    const int end = bvh_build_rec(B, cen, first + half, count - half, right);
    /* children stored as (left, right) indices: left = node + 1 always */
    nd = &B->nodes[node];
    nd->first = right;
    nd->count = 0;
    return end;
}

void *orc_bvh_build(const rt_scene_desc *sc) {
    orc_bvh *B = (orc_bvh *)calloc(1, sizeof *B);
    if (!B) return NULL;
    B->mt = sc->mesh_triangle_total;
    B->ns = sc->sphere_count;
    B->n = B->mt + B->ns + sc->triangle_count;
    B->mesh_count = sc->mesh_count;
    const int n = B->n > 0 ? B->n : 1;
    B->prim = (int *)malloc(sizeof(int) * (size_t)n);
    B->mesh_of = (int *)malloc(sizeof(int) * (size_t)n);
    B->plo = (float *)malloc(sizeof(float) * 3 * (size_t)n);
    B->phi = (float *)malloc(sizeof(float) * 3 * (size_t)n);
    float *cen = (float *)malloc(sizeof(float) * 3 * (size_t)n);
    B->nodes = (bnode *)malloc(sizeof(bnode) * 2 * (size_t)n);
    rt_aabb box;
    orc_scene_aabb(sc, &box);
    float scale = 0.0f;
    for (int a = 0; a < 3; ++a) scale = fmaxf(scale, fabsf(comp(box.min, a)) + fabsf(comp(box.max, a)));
    const float pad_abs = ldexpf(fmaxf(scale, 1e-30f), -13);
    for (int m = 0; m < sc->mesh_count; ++m)
        for (int i = 0; i < sc->meshes[m].triangle_count; ++i) B->mesh_of[sc->meshes[m].first_triangle + i] = m;
    for (int r = 0; r < B->n; ++r) {
        float lo[3], hi[3];
        if (r >= B->mt && r < B->mt + B->ns) {
            const rt_sphere sp = sc->spheres[r - B->mt];
            const float rad = sqrtf(sp.radius_squared);
            for (int a = 0; a < 3; ++a) { lo[a] = comp(sp.center, a) - rad; hi[a] = comp(sp.center, a) + rad; }
        } else {
            const rt_triangle t = r < B->mt ? sc->mesh_triangles[r] : sc->triangles[r - B->mt - B->ns];
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(comp(t.vertex0, a), fminf(comp(t.vertex1, a), comp(t.vertex2, a)));
                hi[a] = fmaxf(comp(t.vertex0, a), fmaxf(comp(t.vertex1, a), comp(t.vertex2, a)));
            }
        }
        float ext = 0.0f;
        for (int a = 0; a < 3; ++a) ext = fmaxf(ext, hi[a] - lo[a]);
        const float pad = pad_abs + ext * 1e-4f;
        for (int a = 0; a < 3; ++a) {
            cen[3 * r + a] = 0.5f * (lo[a] + hi[a]);
            B->plo[3 * r + a] = lo[a] - pad;
            B->phi[3 * r + a] = hi[a] + pad;
        }
        B->prim[r] = r;
    }
    B->nnodes = B->n > 0 ? bvh_build_rec(B, cen, 0, B->n, 0) : 0;
    free(cen);
    return B;
}

void orc_bvh_free(void *h) {
    orc_bvh *B = (orc_bvh *)h;
    if (!B) return;
    free(B->prim); free(B->mesh_of); free(B->plo); free(B->phi); free(B->nodes);
    free(B);
}

/* per-thread mesh-gate cache: gate[m] holds (ray stamp << 1 | result) */
static _Thread_local unsigned long long *t_gate;
static _Thread_local int t_gate_n;
static _Thread_local unsigned long long t_stamp;

static rt_hit bvh_intersect(const orc_bvh *B, const rt_scene_desc *sc, const rt_aabb *scene_box,
                            const rt_ray *ray, orc_tests *ct) {
    rt_hit hit;
    hit.type = 0; hit.index = -1; hit.mesh_index = -1;
    hit.distance = FLT_MAX;
    ct->box++;
    if (B->n == 0 || !orc_ray_aabb(ray, scene_box)) return hit; /* Scene.cs:54 */
    if (t_gate_n < B->mesh_count) {
        free(t_gate);
        t_gate = (unsigned long long *)calloc((size_t)B->mesh_count, sizeof *t_gate);
        t_gate_n = B->mesh_count;
    }
    const unsigned long long stamp = ++t_stamp;
    const float o[3] = {ray->origin.x, ray->origin.y, ray->origin.z};
    const float inv[3] = {1.0f / ray->direction.x, 1.0f / ray->direction.y, 1.0f / ray->direction.z};
    float best = FLT_MAX;
    int best_rank = 0x7fffffff;
    int stack[128];
    int sp = 0;
    int node = 0;
    for (;;) {
        const bnode *nd = &B->nodes[node];
        float tn = 0.0f, tf = INFINITY;
        for (int a = 0; a < 3; ++a) { /* conservative slab (padded box); NaN operands ignored */
            const float t1 = (nd->lo[a] - o[a]) * inv[a], t2 = (nd->hi[a] - o[a]) * inv[a];
            tn = fmaxf(tn, fminf(t1, t2));
            tf = fminf(tf, fmaxf(t1, t2));
        }
        const int enter = tn <= tf && tn <= best;
        if (enter && nd->count > 0) {
            for (int i = nd->first; i < nd->first + nd->count; ++i) {
                const int r = B->prim[i];
                float t;
                int ok;
                if (r < B->mt) {
                    const int m = B->mesh_of[r];
                    unsigned long long g = t_gate[m];
                    if ((g >> 1) != stamp) { /* Mesh.AABB gate, Scene.cs:67, once per ray and mesh */
                        ct->box++;
                        g = (stamp << 1) | (unsigned long long)(orc_ray_aabb(ray, &sc->meshes[m].aabb) != 0);
                        t_gate[m] = g;
                    }
                    if (!(g & 1)) continue;
                    ct->tri++;
                    ok = orc_ray_triangle(ray, &sc->mesh_triangles[r], &t);
                } else if (r < B->mt + B->ns) {
                    ct->sph++;
                    ok = orc_ray_sphere(ray, &sc->spheres[r - B->mt], &t);
                } else {
                    ct->tri++;
                    ok = orc_ray_triangle(ray, &sc->triangles[r - B->mt - B->ns], &t);
                }
                if (ok && (t < best || (t == best && r < best_rank))) {
                    best = t;
                    best_rank = r;
                }
            }
        } else if (enter) {
            stack[sp++] = nd->first; /* right child after the left (node + 1) */
            node = node + 1;
            continue;
        }
        if (sp == 0) break;
        node = stack[--sp];
    }
    if (best_rank != 0x7fffffff) {
        hit.distance = best;
        if (best_rank < B->mt) {
            const int m = B->mesh_of[best_rank];
            hit.type = 3; hit.mesh_index = m; hit.index = best_rank - sc->meshes[m].first_triangle;
        } else if (best_rank < B->mt + B->ns) {
            hit.type = 1; hit.index = best_rank - B->mt;
        } else {
            hit.type = 2; hit.index = best_rank - B->mt - B->ns;
        }
    }
    return hit;
}

/* ------------------------------------------------------------------------
 * The GPU's own 4-wide BVH (rt_export_bvh: the records exactly as they lie
 * in HBM, unity-raytracer_amd/csrc/rt_device.h) traversed on the CPU — the
 * CPU-baseline leg that runs the very tree the GPU runs, so the split between
 * the algorithm's speed-up and the hardware's is like for like.  Per ray, as
 * the GPU's per-lane traversal (csrc/traverse.h): the exact scene gate, then
 * near-first closest hit over the padded node boxes (ties to the lowest
 * reference rank), the exact Mesh.AABB gate per leaf (Scene.cs:67), and
 * shadow rays as any-hit queries with the predicate t*t < d2.  Same answers as
 * the brute-force scan (the GPU parity tests hold that for this tree).
 *
 * The walk restates the GPU's per-lane traversal step for step
 * (unity-raytracer_amd/csrc/traverse.h trav_step, as the counting launch
 * RT_FLAG_COUNT_TESTS runs it): the exact node test (plane - o) * (1/d) per
 * child (child_key_exact), the children ordered by the same five-comparator
 * network on their entry distances (misses = +inf; closest-hit and any-hit
 * queries alike), the hit ones pushed far-first, triangle leaves tested in
 * order with an early exit on an occluder, and the mesh gate re-evaluated
 * whenever a leaf of another mesh than the last evaluated one is reached.  So
 * its box / triangle / sphere / shading counts are the canonical counts
 * SURVEY §8(d) prices, and the GPU counting launch must reproduce them
 * exactly (tests/test_gpu_counts.py).
 * --------------------------------------------------------------------- */
typedef struct { float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4]; int32_t child[4], pad[4]; } orc_node4;
typedef struct { float p0[4], p1[4], p2[4]; } orc_trirec;  /* v0 e1.x | e1.yz e2.xy | e2.z rank gate - */
typedef struct { float cr[4]; int32_t misc[4]; } orc_sphrec;  /* center r2 | rank gate - - */

typedef struct orc_bvh4 {
    orc_node4 *nodes;
    orc_trirec *tris;
    orc_sphrec *sphs;
    int nnodes, ntris, nsphs, mt, ns, mesh_count;
    int *mesh_of; /* rank -> mesh (mesh triangles) */
} orc_bvh4;

static inline int rbits(float f) { int i; memcpy(&i, &f, 4); return i; }

void *orc_bvh4_create(const rt_scene_desc *sc, const void *nodes, int32_t nnodes, const void *tris, int32_t ntris,
                      const void *sphs, int32_t nsphs) {
    orc_bvh4 *B = (orc_bvh4 *)calloc(1, sizeof *B);
    if (!B) return NULL;
    B->nnodes = nnodes; B->ntris = ntris; B->nsphs = nsphs;
    B->mt = sc->mesh_triangle_total; B->ns = sc->sphere_count; B->mesh_count = sc->mesh_count;
    B->nodes = (orc_node4 *)malloc(sizeof(orc_node4) * (size_t)(nnodes > 0 ? nnodes : 1));
    B->tris = (orc_trirec *)malloc(sizeof(orc_trirec) * (size_t)(ntris > 0 ? ntris : 1));
    B->sphs = (orc_sphrec *)malloc(sizeof(orc_sphrec) * (size_t)(nsphs > 0 ? nsphs : 1));
    B->mesh_of = (int *)malloc(sizeof(int) * (size_t)(B->mt > 0 ? B->mt : 1));
    if (nnodes) memcpy(B->nodes, nodes, sizeof(orc_node4) * (size_t)nnodes);
    if (ntris) memcpy(B->tris, tris, sizeof(orc_trirec) * (size_t)ntris);
    if (nsphs) memcpy(B->sphs, sphs, sizeof(orc_sphrec) * (size_t)nsphs);
    for (int m = 0; m < sc->mesh_count; ++m)
        for (int i = 0; i < sc->meshes[m].triangle_count; ++i) B->mesh_of[sc->meshes[m].first_triangle + i] = m;
    return B;
}

void orc_bvh4_free(void *h) {
    orc_bvh4 *B = (orc_bvh4 *)h;
    if (!B) return;
    free(B->nodes); free(B->tris); free(B->sphs); free(B->mesh_of);
    free(B);
}

/* One query.  any: shadow ray, true when some primitive has t*t < d2 (node
 * culling at tlimit); otherwise the closest hit (best, best_rank). */
static int bvh4_query(const orc_bvh4 *B, const rt_scene_desc *sc, const rt_aabb *scene_box, const rt_ray *ray,
                      int any, float tlimit, float d2, float *best_out, int *rank_out, orc_tests *ct) {
    *best_out = FLT_MAX;
    *rank_out = -1;
    ct->box++;
    if (B->nnodes == 0 || !orc_ray_aabb(ray, scene_box)) return 0; /* Scene.cs:54 */
    int gate_cached = -1, gate_ok = 0; /* the last mesh whose gate was evaluated (traverse.h Trav) */
    const float o[3] = {ray->origin.x, ray->origin.y, ray->origin.z};
    const float inv[3] = {1.0f / ray->direction.x, 1.0f / ray->direction.y, 1.0f / ray->direction.z};
    float best = FLT_MAX, cull = any ? tlimit : FLT_MAX;
    int best_rank = 0x7fffffff;
    int stack[256], sp = 0, ref = 0;
    for (;;) {
        if (ref >= 0) {
            const orc_node4 *nd = &B->nodes[ref];
            const float *lo[3] = {nd->lox, nd->loy, nd->loz}, *hi[3] = {nd->hix, nd->hiy, nd->hiz};
            float key[4];
            int ch[4];
            for (int c = 0; c < 4; ++c) { /* child_key_exact: padded box; NaN operands ignored */
                float t1[3], t2[3];
                for (int a = 0; a < 3; ++a) {
                    t1[a] = (lo[a][c] - o[a]) * inv[a];
                    t2[a] = (hi[a][c] - o[a]) * inv[a];
                }
                const float tn = fmaxf(fmaxf(fminf(t1[0], t2[0]), fminf(t1[1], t2[1])), fmaxf(fminf(t1[2], t2[2]), 0.0f));
                const float tf = fminf(fminf(fmaxf(t1[0], t2[0]), fmaxf(t1[1], t2[1])), fminf(fmaxf(t1[2], t2[2]), cull));
                ct->box++;
                key[c] = tn <= tf ? tn : INFINITY;
                ch[c] = nd->child[c];
            }
            /* the GPU's sorting network (traverse.h RT_CSWAP order), swap iff k[j] < k[i] */
            static const int net[5][2] = {{0, 1}, {2, 3}, {0, 2}, {1, 3}, {1, 2}};
            for (int s = 0; s < 5; ++s) {
                const int i = net[s][0], j = net[s][1];
                if (key[j] < key[i]) {
                    const float tk = key[i]; key[i] = key[j]; key[j] = tk;
                    const int tc = ch[i]; ch[i] = ch[j]; ch[j] = tc;
                }
            }
            if (key[0] == INFINITY) goto pop;
            const int nh = 1 + (key[1] != INFINITY) + (key[2] != INFINITY) + (key[3] != INFINITY);
            for (int k = nh - 1; k >= 1; --k) stack[sp++] = ch[k];
            ref = ch[0];
            continue;
        } else {
            const int v = ~ref, first = v & ((1 << 27) - 1), count = ((v >> 27) & 3) + 1, kind = (v >> 29) & 1;
            for (int i = first; i < first + count; ++i) {
                float t;
                int ok, rank;
                if (kind == 0) {
                    const orc_trirec *r = &B->tris[i];
                    const int gate = rbits(r->p2[2]);
                    rank = rbits(r->p2[1]);
                    if (gate >= 0) {
                        if (gate != gate_cached) { /* Mesh.AABB gate, Scene.cs:67 */
                            ct->box++;
                            gate_cached = gate;
                            gate_ok = orc_ray_aabb(ray, &sc->meshes[gate].aabb) != 0;
                        }
                        if (!gate_ok) continue;
                    }
                    ct->tri++;
                    /* RMath.RayTriangleIntersection :29-73 on the stored edges (v1 - v0, v2 - v0) */
                    const f3 d = ray->direction, v0 = V(r->p0[0], r->p0[1], r->p0[2]);
                    const f3 e1 = V(r->p0[3], r->p1[0], r->p1[1]), e2 = V(r->p1[2], r->p1[3], r->p2[0]);
                    const f3 h = cross(d, e2);
                    const float a = dot(e1, h);
                    if (a > -RMATH_EPSILON && a < RMATH_EPSILON) continue;
                    const float f = 1.0f / a;
                    const f3 sv = sub(ray->origin, v0);
                    const float u = f * dot(sv, h);
                    if (u < 0.0f || u > 1.0f) continue;
                    const f3 q = cross(sv, e1);
                    const float vv = f * dot(d, q);
                    if (vv < 0.0f || u + vv > 1.0f) continue;
                    t = f * dot(e2, q);
                    ok = t > RMATH_EPSILON;
                } else {
                    const orc_sphrec *r = &B->sphs[i];
                    rt_sphere sp2;
                    sp2.center = V(r->cr[0], r->cr[1], r->cr[2]);
                    sp2.radius_squared = r->cr[3];
                    rank = r->misc[0];
                    ct->sph++;
                    ok = orc_ray_sphere(ray, &sp2, &t);
                }
                if (!ok) continue;
                if (any) {
                    if (t * t < d2) { *rank_out = 1; return 1; }
                } else if (t < best || (t == best && rank < best_rank)) {
                    best = t;
                    best_rank = rank;
                    cull = t;
                }
            }
        }
    pop:
        if (sp == 0) break;
        ref = stack[--sp];
    }
    if (!any && best_rank != 0x7fffffff) {
        *best_out = best;
        *rank_out = best_rank;
    }
    return *rank_out >= 0;
}

static rt_hit bvh4_intersect(const orc_bvh4 *B, const rt_scene_desc *sc, const rt_aabb *scene_box,
                             const rt_ray *ray, orc_tests *ct) {
    rt_hit hit;
    hit.type = 0; hit.index = -1; hit.mesh_index = -1;
    hit.distance = FLT_MAX;
    float best;
    int r;
    if (!bvh4_query(B, sc, scene_box, ray, 0, 0.0f, 0.0f, &best, &r, ct)) return hit;
    hit.distance = best;
    if (r < B->mt) {
        const int m = B->mesh_of[r];
        hit.type = 3; hit.mesh_index = m; hit.index = r - sc->meshes[m].first_triangle;
    } else if (r < B->mt + B->ns) {
        hit.type = 1; hit.index = r - B->mt;
    } else {
        hit.type = 2; hit.index = r - B->mt - B->ns;
    }
    return hit;
}

typedef struct {
    const rt_scene_desc *sc;
    rt_aabb scene_box;
    f3 bg255;          /* new Rgb(BackgroundColor) = float3(r,g,b) * 255f, Rgb.cs:15-18 */
    int max_bounces;
    const orc_bvh *bvh; /* null: the reference's brute-force scan */
    const orc_bvh4 *bvh4; /* non-null: the GPU's tree (closest hits; shadow rays any-hit) */
} frame_t;

static rt_hit trace(const frame_t *fr, const rt_ray *ray, orc_tests *ct) {
    if (fr->bvh4) return bvh4_intersect(fr->bvh4, fr->sc, &fr->scene_box, ray, ct);
    return fr->bvh ? bvh_intersect(fr->bvh, fr->sc, &fr->scene_box, ray, ct)
                   : intersect(fr->sc, &fr->scene_box, ray, ct);
}

/* RayTracingSetup.CalculateSpecular, :375-400 */
static f3 calc_specular(f3 light_dir, f3 ray_dir, f3 n, f3 ks, f3 irr, float phong) {
    float ldn = dot(light_dir, n);
    float angle = degrees(uacos(ldn));
    if (angle > 90.0f) return V(0.0f, 0.0f, 0.0f);
    f3 v = add(light_dir, ray_dir);
    f3 halfway = divs(v, length(v));
    float c = umax(0.0f, dot(n, halfway));
    return mul(muls(ks, upow(c, phong)), irr);
}

/* RayTracingSetup.Shade, :304-366 (literal recursion) */
static f3 shade(const frame_t *fr, rt_ray ray, int bounce, orc_counts *cnt) {
    orc_tests ct = {0, 0, 0};
    rt_hit hit = trace(fr, &ray, &ct);
    if (hit.type == 0) {
        cnt->box_tests += ct.box; cnt->triangle_tests += ct.tri; cnt->sphere_tests += ct.sph;
        return fr->bg255;
    }
    const rt_scene_desc *sc = fr->sc;
    /* Ray.GetPoint, Ray.cs:18-21 */
    f3 p = add(ray.origin, muls(ray.direction, hit.distance));
    /* GetSurfaceNormalAndMaterial, :409-436 */
    f3 n;
    const rt_material *mat;
    if (hit.type == 1) {
        n = normalize(sub(p, sc->spheres[hit.index].center)); /* GetSphereNormal :402-407 */
        mat = &sc->sphere_materials[hit.index];
    } else if (hit.type == 2) {
        n = sc->triangle_normals[hit.index];
        mat = &sc->triangle_materials[hit.index];
    } else {
        const rt_mesh *mesh = &sc->meshes[hit.mesh_index];
        n = sc->mesh_triangle_normals[mesh->first_triangle + hit.index];
        mat = &mesh->material;
    }
    cnt->shading_fetches++;
    /* CalculateAmbient :438-441: ambientRadiance * ambientReflectance */
    f3 color = mul(sc->ambient_radiance, mat->ambient_reflectance);
    f3 ray_dir = normalize(sub(ray.origin, p));
    for (int l = 0; l < sc->point_light_count; ++l) {
        const rt_point_light *pl = &sc->point_lights[l];
        f3 light_dir = normalize(sub(pl->position, p));
        rt_ray shadow;
        shadow.origin = add(p, muls(n, SHADOW_RAY_EPSILON));
        shadow.direction = light_dir;
        cnt->shadow_rays++;
        float light_dist_sq = distancesq(p, pl->position);
        if (fr->bvh4) { /* any-hit on the GPU's tree: the same predicate (t >= 0, so t*t is monotone) */
            float bt;
            int br;
            if (bvh4_query(fr->bvh4, sc, &fr->scene_box, &shadow, 1, sqrtf(light_dist_sq) * 1.001f, light_dist_sq, &bt,
                           &br, &ct))
                continue;
        } else {
            rt_hit sh = trace(fr, &shadow, &ct);
            if (sh.type != 0) {
                float hd2 = sh.distance * sh.distance;
                if (hd2 < light_dist_sq) continue;
            }
        }
        f3 irr = divs(pl->intensity, light_dist_sq);
        /* CalculateDiffuse :443-455: diffuse * max(0, dot(L, N)) * E */
        float cosl = umax(0.0f, dot(light_dir, n));
        f3 diffuse = mul(muls(mat->diffuse_reflectance, cosl), irr);
        f3 specular = calc_specular(light_dir, ray_dir, n, mat->specular_reflectance, irr,
                                    mat->phong_exponent);
        color = add(color, add(diffuse, specular));
    }
    cnt->box_tests += ct.box; cnt->triangle_tests += ct.tri; cnt->sphere_tests += ct.sph;
    if (mat->is_mirror && bounce < fr->max_bounces) {
        /* Reflect :368-373: origin P + N*eps, dir (2*N)*dot(V,N) - V (not renormalised) */
        rt_ray refl;
        refl.origin = add(p, muls(n, SHADOW_RAY_EPSILON));
        refl.direction = sub(muls(smul(2.0f, n), dot(ray_dir, n)), ray_dir);
        cnt->reflection_rays++;
        f3 sub_color = shade(fr, refl, bounce + 1, cnt);
        color = add(color, mul(mat->mirror_reflectance, sub_color));
    }
    return color;
}

static int isqrt_exact(int v) {
    if (v <= 0) return -1;
    int n = 1;
    while (n * n < v) ++n;
    return n * n == v ? n : -1;
}

/* One pixel: CastPixelRays :288-300 with the n*n stratified extension
 * (n == 1 reproduces the reference's fixed 0.5 offsets bit for bit). */
static void pixel(const frame_t *fr, const rt_camera *cam, f3 top_left, float hl, float vl,
                  int res_x, int res_y, int n, int x, int y, float *out4, orc_counts *cnt) {
    f3 sum = V(0, 0, 0);
    for (int sj = 0; sj < n; ++sj) {
        float oy = ((float)sj + 0.5f) / (float)n;
        for (int si = 0; si < n; ++si) {
            float ox = ((float)si + 0.5f) / (float)n;
            float right_move = (((float)x + ox) * hl) / (float)res_x;
            float down_move = (((float)y + oy) * vl) / (float)res_y;
            f3 pix = sub(add(top_left, smul(right_move, cam->right)), muls(cam->up, down_move));
            rt_ray ray;
            ray.origin = cam->position;
            ray.direction = normalize(sub(pix, cam->position));
            cnt->primary_rays++;
            f3 c = shade(fr, ray, 0, cnt);
            sum = (sj == 0 && si == 0) ? c : add(sum, c);
        }
    }
    float inv_n2 = (float)(n * n);
    if (n > 1) sum = divs(sum, inv_n2);
    /* Rgb.Color, Rgb.cs:13: Value / 255f, alpha 1 */
    out4[0] = sum.x / 255.0f;
    out4[1] = sum.y / 255.0f;
    out4[2] = sum.z / 255.0f;
    out4[3] = 1.0f;
}

static int setup(frame_t *fr, const rt_scene_desc *sc, const rt_image_plane *plane,
                 const rt_render_params *prm, int *n_out) {
    if (!sc || !plane || !prm) return RT_E_INVALID;
    int n = isqrt_exact(prm->samples_per_pixel);
    if (n < 0) return RT_E_INVALID;
    fr->sc = sc;
    fr->bvh = NULL;
    fr->bvh4 = NULL;
    orc_scene_aabb(sc, &fr->scene_box);
    fr->bg255 = muls(V(prm->background_color[0], prm->background_color[1], prm->background_color[2]), 255.0f);
    fr->max_bounces = prm->max_reflection_bounces;
    *n_out = n;
    return RT_OK;
}

/* ImagePlane.GetRect(...).TopLeft, ImagePlane.cs:26-44 */
static f3 top_left_of(const rt_camera *cam, const rt_image_plane *plane) {
    f3 center = add(cam->position, muls(cam->forward, plane->distance_to_camera));
    f3 half_up = muls(cam->up, plane->half_vertical_length);
    f3 half_right = muls(cam->right, plane->half_horizontal_length);
    return add(sub(center, half_right), half_up);
}

/* Render the pixels listed in pix_idx (x + y*res_x) into out (4 floats each). */
static int render_pixels(const orc_bvh *bvh, const orc_bvh4 *bvh4, const rt_scene_desc *sc, const rt_camera *cam,
                         const rt_image_plane *plane, const rt_render_params *prm, const int32_t *pix_idx,
                         int32_t npix, float *out, orc_counts *counts, int32_t threads);

int orc_render_pixels(const rt_scene_desc *sc, const rt_camera *cam, const rt_image_plane *plane,
                      const rt_render_params *prm, const int32_t *pix_idx, int32_t npix,
                      float *out, orc_counts *counts, int32_t threads) {
    return render_pixels(NULL, NULL, sc, cam, plane, prm, pix_idx, npix, out, counts, threads);
}

/* The same pixels through the GPU's own 4-wide BVH (orc_bvh4_create). */
int orc_render_pixels_bvh4(const void *bvh4, const rt_scene_desc *sc, const rt_camera *cam,
                           const rt_image_plane *plane, const rt_render_params *prm, const int32_t *pix_idx,
                           int32_t npix, float *out, orc_counts *counts, int32_t threads) {
    return render_pixels(NULL, (const orc_bvh4 *)bvh4, sc, cam, plane, prm, pix_idx, npix, out, counts, threads);
}

/* The same pixels with closest hits through a CPU BVH (orc_bvh_build over sc). */
int orc_render_pixels_bvh(const void *bvh, const rt_scene_desc *sc, const rt_camera *cam,
                          const rt_image_plane *plane, const rt_render_params *prm, const int32_t *pix_idx,
                          int32_t npix, float *out, orc_counts *counts, int32_t threads) {
    return render_pixels((const orc_bvh *)bvh, NULL, sc, cam, plane, prm, pix_idx, npix, out, counts, threads);
}

static int render_pixels(const orc_bvh *bvh, const orc_bvh4 *bvh4, const rt_scene_desc *sc, const rt_camera *cam,
                         const rt_image_plane *plane, const rt_render_params *prm, const int32_t *pix_idx,
                         int32_t npix, float *out, orc_counts *counts, int32_t threads) {
    frame_t fr;
    int n;
    int st = setup(&fr, sc, plane, prm, &n);
    if (st) return st;
    fr.bvh = bvh;
    fr.bvh4 = bvh4;
    f3 tl = top_left_of(cam, plane);
    float hl = plane->half_horizontal_length * 2.0f; /* HorizontalLength, ImagePlane.cs:23 */
    float vl = plane->half_vertical_length * 2.0f;
    int res_x = plane->resolution_x, res_y = plane->resolution_y;
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0;
    if (threads < 1) threads = 1;
#pragma omp parallel for schedule(dynamic, 16) num_threads(threads) \
    reduction(+ : c0, c1, c2, c3, c4, c5, c6)
    for (int32_t k = 0; k < npix; ++k) {
        orc_counts cnt;
        memset(&cnt, 0, sizeof cnt);
        int32_t idx = pix_idx[k];
        pixel(&fr, cam, tl, hl, vl, res_x, res_y, n, idx % res_x, idx / res_x, out + 4 * (size_t)k, &cnt);
        c0 += cnt.primary_rays; c1 += cnt.shadow_rays; c2 += cnt.reflection_rays;
        c3 += cnt.box_tests; c4 += cnt.triangle_tests; c5 += cnt.sphere_tests; c6 += cnt.shading_fetches;
    }
    if (counts) {
        counts->primary_rays = c0; counts->shadow_rays = c1; counts->reflection_rays = c2;
        counts->box_tests = c3; counts->triangle_tests = c4; counts->sphere_tests = c5;
        counts->shading_fetches = c6;
    }
    return RT_OK;
}

/* Whole frame (PixelColors, index x + y*res_x), rows y0..y1-1 only when
 * row_step > 1 is used for sub-sampled CPU baselines. */
int orc_render_rows(const rt_scene_desc *sc, const rt_camera *cam, const rt_image_plane *plane,
                    const rt_render_params *prm, int32_t row_start, int32_t row_step,
                    float *out, orc_counts *counts, int32_t threads) {
    if (!plane) return RT_E_INVALID;
    int res_x = plane->resolution_x, res_y = plane->resolution_y;
    if (res_x < 0 || res_y < 0 || row_step < 1 || row_start < 0) return RT_E_INVALID;
    int32_t nrows = row_start < res_y ? (res_y - row_start + row_step - 1) / row_step : 0;
    int32_t npix = nrows * res_x;
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(npix > 0 ? npix : 1));
    if (!idx) return RT_E_INTERNAL;
    int32_t k = 0;
    for (int32_t r = 0; r < nrows; ++r)
        for (int32_t x = 0; x < res_x; ++x) idx[k++] = (row_start + r * row_step) * res_x + x;
    int st = orc_render_pixels(sc, cam, plane, prm, idx, npix, out, counts, threads);
    free(idx);
    return st;
}

int orc_render(const rt_scene_desc *sc, const rt_camera *cam, const rt_image_plane *plane,
               const rt_render_params *prm, float *out, orc_counts *counts, int32_t threads) {
    return orc_render_rows(sc, cam, plane, prm, 0, 1, out, counts, threads);
}

/* The specular back-face decision `degrees(acos(d)) > 90f` (:384-392) as the
 * oracle evaluates it, exported so tests can pin the GPU's threshold form. */
int orc_spec_backfacing(float d) { return degrees(uacos(d)) > 90.0f; }
