// RayTracingSetupNative.cs — RayTracingSetup with its per-frame trace
// (CastPixelRays, RayTracingSetup.cs:275-302) and scene extraction
// (UpdateScene :120-128, SceneMesh.Mesh SceneMesh.cs:11-53) moved to the
// MI355X library.  SOURCE ONLY (no Mono/Unity in the build image).
//
// Per frame the component uploads only what changed:
//   * every field the reference's Fetch* methods read is re-read each Update
//     (as the reference does) and compared byte for byte with the last copy;
//     any change re-sends the scene source (rt_set_scene_source);
//   * otherwise only the localToWorld matrices (rt_update_mesh_transforms,
//     64 B per mesh) — extraction and the BVH refit run on the GPU.
// PixelColors keeps the reference's Color[] (float RGBA, RT_FLAG_OUT default);
// set OutputRgba8 to receive Color32[] for a Texture2D instead (4x fewer
// bytes over PCIe).
using System;
using System.Collections.Generic;
using System.Linq;
using System.Runtime.InteropServices;
using Unity.Mathematics;
// MemoryMarshal / ReadOnlySpan: .NET Standard 2.1 (Unity 2021.3)
using UnityEngine;

namespace RayTracer.Native
{
    public class RayTracingSetupNative : MonoBehaviour
    {
        public ImagePlane ImagePlane;
        public Color BackgroundColor = Color.black;
        public int MaxReflectionBounces = 1;
        public int SamplesPerPixel = 1;          // n*n; 1 == the reference
        public bool OutputRgba8;
        public int NumGpus = 1;                  // > 1: row bands on that many GPUs, gathered to GPU 0 in the library

        public Color[] PixelColors = Array.Empty<Color>();
        public Color32[] PixelColors32 = Array.Empty<Color32>();
        public RtStats LastStats;

        IntPtr _rt;
        RtMatrix[] _matrices = Array.Empty<RtMatrix>();

        void Start()
        {
            if (Rt.rt_create(out _rt, NumGpus) != Rt.OK)
                Debug.LogError(Rt.LastError(IntPtr.Zero));
        }

        void OnDestroy()
        {
            if (_rt != IntPtr.Zero) Rt.rt_destroy(_rt);
            _rt = IntPtr.Zero;
        }

        void Update()
        {
            if (_rt == IntPtr.Zero) return;
            var cam = Camera.main;
            var cameraData = new CameraData
            {
                Position = cam.transform.position,
                Forward = math.normalize(cam.transform.forward),
                Right = math.normalize(cam.transform.right),
                Up = math.normalize(cam.transform.up),
            };
            UpdateScene();
            CastPixelRays(cameraData);
        }

        // UpdateScene (:120-128).  Every Update re-reads exactly what the
        // reference's Fetch* methods read (FetchTriangles :159-169 -> SceneTriangle
        // position + Offset0/1/2 + Material; FetchSpheres -> SceneSphere position,
        // localScale.x, Material; FetchMeshes -> SceneMesh sharedMesh, vertices,
        // triangles, localToWorldMatrix, Material; FetchPointLights ->
        // ScenePointLight position + Intensity; FetchAmbientLights ->
        // SceneAmbientLight.AmbientLight) and compares it byte for byte with the
        // previous Update's copy; on any difference the whole scene source is
        // re-sent (rt_set_scene_source), otherwise only the mesh matrices
        // (rt_update_mesh_transforms: device extraction + BVH rebuild).
        // DetectMeshEdits = false skips re-reading Mesh.vertices / triangles
        // (the one read whose cost grows with the mesh, as in the reference):
        // then an in-place edit of a shared mesh's vertex or index buffer is
        // NOT seen — Unity keeps no cheap version counter on a Mesh.
        public bool DetectMeshEdits = true;

        StaticScene _static;

        struct StaticScene
        {
            public Triangle[] Tris;
            public RtMaterial[] TriMats, SphMats, MeshMats;
            public Sphere[] Spheres;
            public PointLightData[] Lights;
            public float3 Ambient;
            public int AmbientCount;
            public SceneMesh[] Meshes;
            public UnityEngine.Mesh[] SharedMeshes;
            public Vector3[][] Vertices;
            public int[][] Indices;
        }

        void UpdateScene()
        {
            var meshes = FindObjectsOfType<SceneMesh>();
            var tris = FindObjectsOfType<SceneTriangle>();
            var spheres = FindObjectsOfType<SceneSphere>();
            var lights = FindObjectsOfType<ScenePointLight>();
            var ambient = FindObjectsOfType<SceneAmbientLight>();
            if (ambient.Length > 1) Debug.LogError("There are more than Single Ambient Lights in the Scene.");

            var cur = new StaticScene
            {
                Tris = tris.Select(t => t.Triangle).ToArray(),
                TriMats = tris.Select(t => Rt.Material(t.Material)).ToArray(),
                Spheres = spheres.Select(x => x.Sphere).ToArray(),
                SphMats = spheres.Select(x => Rt.Material(x.Material)).ToArray(),
                Lights = lights.Select(l => l.Light).ToArray(),
                // FetchAmbientLights (:130-147): more than one -> logged, none used
                Ambient = ambient.Length == 1 ? ambient[0].AmbientLight.Radiance : float3.zero,
                AmbientCount = ambient.Length,
                Meshes = meshes,
                SharedMeshes = meshes.Select(m => m.MeshFilter.sharedMesh).ToArray(),
                MeshMats = meshes.Select(m => Rt.Material(m.Material)).ToArray(),
            };
            if (DetectMeshEdits)
            {
                cur.Vertices = cur.SharedMeshes.Select(m => m.vertices).ToArray();
                cur.Indices = cur.SharedMeshes.Select(m => m.triangles).ToArray();
            }
            if (SameScene(cur, _static))
            {
                for (int i = 0; i < meshes.Length; i++)
                    _matrices[i] = RtMatrix.FromUnity(meshes[i].transform.localToWorldMatrix);
                if (Rt.rt_update_mesh_transforms(_rt, _matrices, _matrices.Length) != Rt.OK)
                    Debug.LogError(Rt.LastError(_rt));
                return;
            }
            SetSceneSource(cur);
            _static = cur;
        }

        // Byte-for-byte equality of two blittable arrays (float bits: a sign
        // of zero or a NaN payload change counts, as it can change the image).
        static bool SameBytes<T>(T[] a, T[] b) where T : unmanaged
        {
            if (a == null || b == null) return a == b;
            return MemoryMarshal.AsBytes(new ReadOnlySpan<T>(a)).SequenceEqual(MemoryMarshal.AsBytes(new ReadOnlySpan<T>(b)));
        }

        static bool SameScene(in StaticScene a, in StaticScene b)
        {
            if (b.Meshes == null) return false;  // first Update
            if (!SameBytes(a.Tris, b.Tris) || !SameBytes(a.TriMats, b.TriMats) || !SameBytes(a.Spheres, b.Spheres) ||
                !SameBytes(a.SphMats, b.SphMats) || !SameBytes(a.Lights, b.Lights) ||
                !SameBytes(new[] { a.Ambient }, new[] { b.Ambient }) || a.AmbientCount != b.AmbientCount ||
                !SameBytes(a.MeshMats, b.MeshMats))
                return false;
            if (!a.Meshes.SequenceEqual(b.Meshes) || !a.SharedMeshes.SequenceEqual(b.SharedMeshes)) return false;
            if (a.Vertices != null)
            {
                if (b.Vertices == null) return false;
                for (int i = 0; i < a.Vertices.Length; i++)
                    if (!SameBytes(a.Vertices[i], b.Vertices[i]) || !SameBytes(a.Indices[i], b.Indices[i]))
                        return false;
            }
            return true;
        }

        void SetSceneSource(in StaticScene sc)
        {
            var handles = new List<GCHandle>();
            IntPtr Pin(Array a)
            {
                if (a.Length == 0) return IntPtr.Zero;
                var h = GCHandle.Alloc(a, GCHandleType.Pinned);
                handles.Add(h);
                return h.AddrOfPinnedObject();
            }
            try
            {
                // FetchTriangles / FetchSpheres / FetchPointLights / FetchAmbientLights
                var desc = new RtSceneDesc
                {
                    Triangles = Pin(sc.Tris),
                    TriangleNormals = Pin(sc.Tris.Select(t => t.Normal).ToArray()),
                    TriangleMaterials = Pin(sc.TriMats),
                    TriangleCount = sc.Tris.Length,
                    Spheres = Pin(sc.Spheres),
                    SphereMaterials = Pin(sc.SphMats),
                    SphereCount = sc.Spheres.Length,
                    PointLights = Pin(sc.Lights),
                    PointLightCount = sc.Lights.Length,
                    AmbientRadiance = sc.Ambient,
                };
                // SceneMesh sources: local vertices + index buffer + transform
                var src = new RtMeshSource[sc.Meshes.Length];
                _matrices = new RtMatrix[sc.Meshes.Length];
                for (int i = 0; i < sc.Meshes.Length; i++)
                {
                    var verts = sc.Vertices != null ? sc.Vertices[i] : sc.SharedMeshes[i].vertices;
                    var idx = sc.Indices != null ? sc.Indices[i] : sc.SharedMeshes[i].triangles;
                    _matrices[i] = RtMatrix.FromUnity(sc.Meshes[i].transform.localToWorldMatrix);
                    src[i] = new RtMeshSource
                    {
                        Vertices = Pin(verts), VertexCount = verts.Length,
                        Indices = Pin(idx), IndexCount = idx.Length,
                        LocalToWorld = _matrices[i], Material = sc.MeshMats[i],
                    };
                }
                // the tree is built once on the host and refitted on the device
                // every Update (rigid per-mesh motion); rebuilt when it degrades
                if (Rt.rt_set_scene_source_ex(_rt, ref desc, src, src.Length, Rt.BuildSahRefit) != Rt.OK)
                    Debug.LogError(Rt.LastError(_rt));
            }
            finally
            {
                foreach (var h in handles) h.Free();
            }
        }

        // CastPixelRays (:275-302)
        void CastPixelRays(CameraData cameraData)
        {
            var plane = new RtImagePlane
            {
                ResX = ImagePlane.Resolution.X, ResY = ImagePlane.Resolution.Y,
                Distance = ImagePlane.DistanceToCamera,
                HalfH = ImagePlane.HalfHorizontalLength, HalfV = ImagePlane.HalfVerticalLength,
            };
            var p = new RtRenderParams
            {
                BgR = BackgroundColor.r, BgG = BackgroundColor.g, BgB = BackgroundColor.b, BgA = 1f,
                MaxBounces = MaxReflectionBounces, Spp = SamplesPerPixel, BandCount = 1, BandRows = 8,
                Flags = OutputRgba8 ? Rt.FlagOutRgba8 : 0,
            };
            int n = plane.ResX * plane.ResY;
            int st;
            if (OutputRgba8)
            {
                if (PixelColors32.Length != n) PixelColors32 = new Color32[n];
                st = Rt.rt_render_rgba8(_rt, ref cameraData, ref plane, ref p, PixelColors32, out LastStats);
            }
            else
            {
                if (PixelColors.Length != n) PixelColors = new Color[n];
                st = Rt.rt_render(_rt, ref cameraData, ref plane, ref p, PixelColors, out LastStats);
            }
            if (st != Rt.OK) Debug.LogError(Rt.LastError(_rt));
        }
    }
}
