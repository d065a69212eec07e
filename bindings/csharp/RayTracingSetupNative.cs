// RayTracingSetupNative.cs — RayTracingSetup with its per-frame trace
// (CastPixelRays, RayTracingSetup.cs:275-302) and scene extraction
// (UpdateScene :120-128, SceneMesh.Mesh SceneMesh.cs:11-53) moved to the
// MI355X library.  SOURCE ONLY (no Mono/Unity in the build image).
//
// Per frame the component uploads only what changed:
//   * mesh vertex/index buffers once (rt_set_scene_source), then the
//     localToWorld matrices every Update (rt_update_mesh_transforms, 64 B per
//     mesh) — extraction and the BVH rebuild run on the GPU;
//   * loose triangles, spheres and lights are re-fetched like the reference
//     (FindObjectsOfType) and, when they change, the scene is re-sent.
// PixelColors keeps the reference's Color[] (float RGBA, RT_FLAG_OUT default);
// set OutputRgba8 to receive Color32[] for a Texture2D instead (4x fewer
// bytes over PCIe).
using System;
using System.Collections.Generic;
using System.Linq;
using System.Runtime.InteropServices;
using Unity.Mathematics;
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
        SceneMesh[] _meshes = Array.Empty<SceneMesh>();
        UnityEngine.Mesh[] _sharedMeshes = Array.Empty<UnityEngine.Mesh>();
        RtMatrix[] _matrices = Array.Empty<RtMatrix>();
        int _staticHash;

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

        // UpdateScene (:120-128): re-send the scene when its object set or a
        // static object changed; otherwise only the mesh transforms.
        void UpdateScene()
        {
            var meshes = FindObjectsOfType<SceneMesh>();
            var tris = FindObjectsOfType<SceneTriangle>();
            var spheres = FindObjectsOfType<SceneSphere>();
            var lights = FindObjectsOfType<ScenePointLight>();
            var ambient = FindObjectsOfType<SceneAmbientLight>();
            if (ambient.Length > 1) Debug.LogError("There are more than Single Ambient Lights in the Scene.");

            int hash = StaticHash(tris, spheres, lights, ambient);
            bool sameMeshes = meshes.Length == _meshes.Length &&
                              meshes.Select(m => m.MeshFilter.sharedMesh).SequenceEqual(_sharedMeshes) &&
                              meshes.SequenceEqual(_meshes);
            if (sameMeshes && hash == _staticHash)
            {
                for (int i = 0; i < meshes.Length; i++)
                    _matrices[i] = RtMatrix.FromUnity(meshes[i].transform.localToWorldMatrix);
                if (Rt.rt_update_mesh_transforms(_rt, _matrices, _matrices.Length) != Rt.OK)
                    Debug.LogError(Rt.LastError(_rt));
                return;
            }
            SetSceneSource(meshes, tris, spheres, lights, ambient.Length == 1 ? ambient[0] : null);
            _staticHash = hash;
        }

        void SetSceneSource(SceneMesh[] meshes, SceneTriangle[] tris, SceneSphere[] spheres,
                            ScenePointLight[] lights, SceneAmbientLight ambient)
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
                var triArr = tris.Select(t => t.Triangle).ToArray();
                var desc = new RtSceneDesc
                {
                    Triangles = Pin(triArr),
                    TriangleNormals = Pin(triArr.Select(t => t.Normal).ToArray()),
                    TriangleMaterials = Pin(tris.Select(t => Rt.Material(t.Material)).ToArray()),
                    TriangleCount = triArr.Length,
                    Spheres = Pin(spheres.Select(s => s.Sphere).ToArray()),
                    SphereMaterials = Pin(spheres.Select(s => Rt.Material(s.Material)).ToArray()),
                    SphereCount = spheres.Length,
                    PointLights = Pin(lights.Select(l => l.Light).ToArray()),
                    PointLightCount = lights.Length,
                    AmbientRadiance = ambient != null ? ambient.AmbientLight.Radiance : float3.zero,
                };
                // SceneMesh sources: local vertices + index buffer + transform
                var src = new RtMeshSource[meshes.Length];
                _sharedMeshes = new UnityEngine.Mesh[meshes.Length];
                _matrices = new RtMatrix[meshes.Length];
                for (int i = 0; i < meshes.Length; i++)
                {
                    var um = meshes[i].MeshFilter.sharedMesh;
                    var verts = um.vertices;
                    var idx = um.triangles;
                    _sharedMeshes[i] = um;
                    _matrices[i] = RtMatrix.FromUnity(meshes[i].transform.localToWorldMatrix);
                    src[i] = new RtMeshSource
                    {
                        Vertices = Pin(verts), VertexCount = verts.Length,
                        Indices = Pin(idx), IndexCount = idx.Length,
                        LocalToWorld = _matrices[i], Material = Rt.Material(meshes[i].Material),
                    };
                }
                _meshes = meshes;
                if (Rt.rt_set_scene_source(_rt, ref desc, src, src.Length) != Rt.OK)
                    Debug.LogError(Rt.LastError(_rt));
            }
            finally
            {
                foreach (var h in handles) h.Free();
            }
        }

        static int StaticHash(SceneTriangle[] t, SceneSphere[] s, ScenePointLight[] l, SceneAmbientLight[] a)
        {
            var h = new HashCode();
            foreach (var x in t) { h.Add(x.GetInstanceID()); h.Add(x.transform.position); }
            foreach (var x in s) { h.Add(x.GetInstanceID()); h.Add(x.transform.position); h.Add(x.transform.localScale); }
            foreach (var x in l) { h.Add(x.GetInstanceID()); h.Add(x.transform.position); h.Add(x.Intensity); }
            foreach (var x in a) h.Add(x.GetInstanceID());
            return h.ToHashCode();
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
