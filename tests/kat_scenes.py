"""Analytic known-answer frames for the shading path.

Every scene is built so that each intermediate value of the reference's
arithmetic is exact in binary32 — the pixel's ray is axis-aligned, divisions
are by powers of two or land on representable values, normals are unit axis
vectors — so the expected Color follows by hand from the C# source alone,
whatever the order of operations, and does not come from either of this
repo's restatements (oracle/rt_oracle.c, oracle/np_oracle.py).  Each expected
value is an exact rational c / 255 (Rgb.Color, Rgb.cs:13-18), rounded once to
float32.  References are to Assets/RayTracer/.

Derivation common to all: a 1x1 image plane at distance 1 with half lengths
0.5 (ImagePlane.cs:23-44): center = pos + fwd; topLeft = (center - right*0.5)
+ up*0.5; for x = y = 0, rm = ((0 + 0.5) * 1) / 1 = 0.5 and dm = 0.5, so the
pixel point is exactly `center` and the ray direction is exactly `fwd`
(CastPixelRays, RayTracingSetup.cs:286-298; normalize of a unit vector).
"""
from fractions import Fraction as Fr

import numpy as np

f32 = np.float32


def color(c):
    """Rgb(c).Color: per channel c / 255 rounded once to float32, alpha 1."""
    return np.array([f32(float(Fr(v) / 255)) for v in c] + [f32(1.0)], f32)


def _mat(rt, kd=(0, 0, 0), ka=(0, 0, 0), km=(0, 0, 0), ks=(0, 0, 0), phong=0.0, mirror=False):
    return rt.MaterialData(DiffuseReflectance=kd, AmbientReflectance=ka, MirrorReflectance=km,
                           SpecularReflectance=ks, PhongExponent=phong, IsMirror=mirror)


def _frame(rt, name, sc, pos, fwd, right, up, bounces=1, bg=(0.0, 0.0, 0.0)):
    S = rt.scenes
    cam = S.CameraData(Position=pos, Forward=fwd, Right=right, Up=up)
    return S.Frame(name, sc, cam, S.ImagePlane(1, 1, 1.0, 0.5, 0.5), background=bg + (1.0,), max_bounces=bounces)


def lit_sphere(rt, intensity=16.0):
    """A6 + A7 + A8 + A9 + A11.  Camera at the origin looking +z; sphere
    c = (0,0,5), r^2 = 1; a point light AT the eye.
    RaySphereIntersection (RMath.cs:81-108): oc = (0,0,-5), uoc = -5,
    disc = 25 - (25 - 1) = 1, sq = 1, small = 4 -> t = 4; P = (0,0,4).
    GetSphereNormal (:402-407): N = normalize(P - c) = (0,0,-1).
    V = normalize(O - P) = (0,0,-1).  Ldir = normalize(L - P) = (0,0,-1),
    d2 = 16, E = I / 16 (:350).  The shadow ray leaves the sphere (origin
    1e-4 outside, moving away: big = -uoc + 1 < 0) -> unoccluded.
    Diffuse (:443-455): kd * max(0, dot(Ldir, N) = 1) * E.
    Specular (:375-400): acos(1) = 0 <= 90; h = (0,0,-2) / 2 = (0,0,-1);
    pow(dot(N, h) = 1, 8) = 1 -> ks * E.  Ambient (:438): radiance * ka.
    I = 16: E = 1 -> c = (4,4,4) + (0.5,0.25,0.125) + (0.25,0.5,0.75).
    I = 16384: E = 1024 -> c > 255: Color is unclamped HDR (Rgb.cs:13)."""
    sc = rt.Scene()
    sc.add_sphere_r2((0.0, 0.0, 5.0), 1.0, _mat(rt, kd=(0.5, 0.25, 0.125), ka=(1.0, 0.5, 0.25),
                                                 ks=(0.25, 0.5, 0.75), phong=8.0))
    sc.add_point_light((0.0, 0.0, 0.0), intensity)
    sc.AmbientLight = np.array((4.0, 8.0, 16.0), f32)
    fr = _frame(rt, f"lit_sphere_{int(intensity)}", sc, (0.0, 0.0, 0.0), (0.0, 0.0, 1.0), (1.0, 0.0, 0.0),
                (0.0, 1.0, 0.0))
    e = Fr(int(intensity), 16)
    c = [Fr(4) + Fr(1, 2) * e + Fr(1, 4) * e, Fr(4) + Fr(1, 4) * e + Fr(1, 2) * e,
         Fr(4) + Fr(1, 8) * e + Fr(3, 4) * e]
    return fr, color(c), (1, 1, 0)  # (primary, shadow, reflection) rays


def mirror_sphere(rt, bounces):
    """A2 (mirror fold) + A10 (Reflect).  Camera and mirror sphere as in
    lit_sphere (no lights); at the sphere N = V = (0,0,-1), so Reflect
    (:368-373) gives ((2N) * dot(V,N)) - V = (0,0,-2) - (0,0,-1) = (0,0,-1):
    straight back, past the eye, onto a loose triangle at z = -4 whose
    Triangle.Normal (Triangle.cs:17-19) is cross(v2-v0, v1-v0) / 4 = (0,0,1).
    Its color (ambient only) is (4,8,16) * (0.25,0.5,1) = (1,4,16).  The mirror's
    own color is 0 (ka = kd = ks = 0), so with MaxReflectionBounces >= 1 the pixel
    is 0 + km * (1,4,16) = (0.5, 1, 12) (Shade :358-363); with 0 it is 0."""
    sc = rt.Scene()
    sc.add_sphere_r2((0.0, 0.0, 5.0), 1.0, _mat(rt, km=(0.5, 0.25, 0.75), mirror=True))
    sc.add_triangles(np.array([[(-1, -1, -4), (0, 1, -4), (1, -1, -4)]], f32), [_mat(rt, ka=(0.25, 0.5, 1.0))])
    sc.AmbientLight = np.array((4.0, 8.0, 16.0), f32)
    fr = _frame(rt, f"mirror_sphere_{bounces}", sc, (0.0, 0.0, 0.0), (0.0, 0.0, 1.0), (1.0, 0.0, 0.0),
                (0.0, 1.0, 0.0), bounces=bounces)
    c = [Fr(1, 2), Fr(1), Fr(12)] if bounces >= 1 else [0, 0, 0]
    return fr, color(c), (1, 0, 1 if bounces >= 1 else 0)


def _floor(rt, sc, mat, y=0.0, mesh=False):
    """Loose floor triangle with v0 = (-8,y,-8), e1 = (16,0,0), e2 = (8,0,16):
    for the ray (0,4,0) -> (0,-1,0), Moller-Trumbore (RMath.cs:29-73) gives
    h = cross(d, e2) = (-16,0,8), a = -256 (1/a exact), s = (8,4-y,8),
    u = 0.25, q = (0,128,-64) (y = 0), v = 0.5, t = 4 - y exactly; the normal
    cross(e2, e1) / 256 = (0,1,0).  mesh=True: the same triangle as a
    SceneMesh with the opposite winding — Mesh.TriangleNormals are
    -Triangle.Normal (SceneMesh.cs:43), so it shades with (0,1,0) too."""
    v = np.array([[(-8, y, -8), (8, y, -8), (0, y, 8)]], f32)
    if mesh:
        v = v[:, [0, 2, 1]]
        sc.add_mesh(rt.Mesh.from_vertices(v.reshape(-1, 3), np.arange(3, dtype=np.int32), mat))
    else:
        sc.add_triangles(v, [mat])


FLOOR_MAT = dict(kd=(0.5, 0.25, 0.125), ka=(1.0, 0.5, 0.25), ks=(0.25, 0.5, 0.75), phong=2.0)


def shadowed_floor(rt, occluder_y):
    """A2 shadow test (RayTracingSetup.cs:329-345) + A5.  Camera at (0,4,0)
    looking down (-y); the floor is hit at t = 4, P = 0, N = V = (0,1,0).
    Light at (0,8,0), I = 64: Ldir = (0,1,0), d2 = 64, E = 1.  An occluding
    triangle at height occluder_y crosses the shadow ray at t ~ occluder_y:
    6 -> t*t = 36 < 64, shadowed: ambient only, (1, 4, 4);
    10 (beyond the light) -> t*t = 100 > 64, not shadowed: ambient + kd*E +
    ks*E = (1.75, 4.75, 4.875) (h = (0,2,0)/2, pow(1, 2) = 1);
    None -> lit as well."""
    sc = rt.Scene()
    _floor(rt, sc, _mat(rt, **FLOOR_MAT))
    if occluder_y is not None:
        y = float(occluder_y)
        sc.add_triangles(np.array([[(-1, y, -1), (1, y, -1), (0, y, 1)]], f32), [_mat(rt)])
    sc.add_point_light((0.0, 8.0, 0.0), 64.0)
    sc.AmbientLight = np.array((1.0, 8.0, 16.0), f32)
    fr = _frame(rt, f"shadowed_floor_{occluder_y}", sc, (0.0, 4.0, 0.0), (0.0, -1.0, 0.0), (1.0, 0.0, 0.0),
                (0.0, 0.0, 1.0))
    amb = [Fr(1), Fr(4), Fr(4)]
    if occluder_y is not None and occluder_y < 8:
        c = amb
    else:
        c = [amb[0] + Fr(1, 2) + Fr(1, 4), amb[1] + Fr(1, 4) + Fr(1, 2), amb[2] + Fr(1, 8) + Fr(3, 4)]
    return fr, color(c), (1, 1, 0)


def tie_floor(rt, mesh_first):
    """A3 ties (Scene.cs:64-115, update only on best > t: the first wins).
    Two coincident floors with different ambient colors, no lights, ambient
    (4,8,16).  mesh_first=False: two loose triangles, the first in
    TriangleData order wins -> ka (0.25,0.5,1) -> (1,4,16).  mesh_first=True:
    the SECOND-listed material sits on a SceneMesh triangle; meshes are
    scanned before loose triangles, so it wins -> ka (1,0.5,0.25) -> (4,4,4);
    the ray also passes the mesh's flat Mesh.AABB gate (t1 = t2 = 4,
    tmin <= tmax, RMath.cs:12-26)."""
    sc = rt.Scene()
    a, b = _mat(rt, ka=(0.25, 0.5, 1.0)), _mat(rt, ka=(1.0, 0.5, 0.25))
    if mesh_first:
        _floor(rt, sc, a)
        _floor(rt, sc, b, mesh=True)
        c = [4, 4, 4]
    else:
        _floor(rt, sc, a)
        _floor(rt, sc, b)
        c = [1, 4, 16]
    sc.AmbientLight = np.array((4.0, 8.0, 16.0), f32)
    fr = _frame(rt, f"tie_floor_{mesh_first}", sc, (0.0, 4.0, 0.0), (0.0, -1.0, 0.0), (1.0, 0.0, 0.0),
                (0.0, 0.0, 1.0))
    return fr, color([Fr(v) for v in c]), (1, 0, 0)


def background(rt):
    """A2 miss (:310-311): the ray misses Scene.AABB; new Rgb(bg).Value is
    bg * 255 = (127.5, 63.75, 31.875) (exact), and .Color divides by 255 again."""
    sc = rt.Scene()
    sc.add_sphere_r2((0.0, 0.0, 5.0), 1.0, _mat(rt, ka=(1.0, 1.0, 1.0)))
    fr = _frame(rt, "background", sc, (0.0, 0.0, 0.0), (0.0, 0.0, -1.0), (-1.0, 0.0, 0.0), (0.0, 1.0, 0.0),
                bg=(0.5, 0.25, 0.125))
    return fr, color([Fr(255, 2), Fr(255, 4), Fr(255, 8)]), (1, 0, 0)


def all_cases(rt):
    return [lit_sphere(rt), lit_sphere(rt, 16384.0), mirror_sphere(rt, 0), mirror_sphere(rt, 1),
            mirror_sphere(rt, 5), shadowed_floor(rt, 6.0), shadowed_floor(rt, 10.0), shadowed_floor(rt, None),
            tie_floor(rt, False), tie_floor(rt, True), background(rt)]
