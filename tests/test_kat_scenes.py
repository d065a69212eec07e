"""Analytic known-answer frames (tests/kat_scenes.py): the CPU oracle must
produce exactly the hand-derived Color (bit for bit) and ray counts; the GPU
library the same through the C-ABI."""
import numpy as np
import pytest

import kat_scenes

NAMES = ["lit_sphere_16", "lit_sphere_16384", "mirror_sphere_0", "mirror_sphere_1", "mirror_sphere_5",
         "shadowed_floor_6.0", "shadowed_floor_10.0", "shadowed_floor_None", "tie_floor_False", "tie_floor_True",
         "background"]


def _case(rt, name):
    cases = {fr.name: (fr, want, rays) for fr, want, rays in kat_scenes.all_cases(rt)}
    assert sorted(cases) == sorted(NAMES)
    return cases[name]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_known_answer(rt, orc, name):
    fr, want, rays = _case(rt, name)
    img, counts = orc.render(fr)
    assert np.array_equal(img[0, 0].view(np.uint32), want.view(np.uint32)), (img[0, 0], want)
    assert (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"]) == rays


@pytest.mark.gpu
@pytest.mark.parametrize("build", [0, 1])
@pytest.mark.parametrize("name", NAMES)
def test_gpu_known_answer(rt, gpu_ctx, name, build):
    fr, want, rays = _case(rt, name)
    gpu_ctx.set_scene(fr.scene, build)
    img, st = gpu_ctx.render(fr.camera, fr.plane, rt.frame_params(fr))
    assert np.array_equal(img[0, 0].view(np.uint32), want.view(np.uint32)), (img[0, 0], want)
    assert (st.primary_rays, st.shadow_rays, st.reflection_rays) == rays
