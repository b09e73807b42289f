"""sampler.RandomSampler (pkg/sampler/random.go:12-57) as a drop-in sampler.

The oracle restates RandomSampler on its own (ORACLE_FLAG_RANDOM_SAMPLER:
Get1D/Get2D straight from the tile's PCG32, no StartPixel draws, Clone's
NewRNGWithSeed + SetSequence). The device renders it as Stratified(ns, 1)
with no sampled dimensions (pbrt_random_sampler, include/pbrt_scene.h); these
tests pin that equivalence bit for bit. No reference test covers
RandomSampler: parity unpinned against Go itself.
"""
import numpy as np
import pytest

import oracle_lib as O
import pbrtgpu as G
from pbrtgpu import abi

ORACLE_FLAG_RANDOM_SAMPLER = 2


def random_desc(ns, **kw):
    rd = abi.render_desc(**kw)
    G.lib().pbrt_random_sampler(ns, G.C.byref(rd))
    return rd


def test_random_sampler_desc():
    rd = random_desc(7, jitter=True, n_dims=4)
    assert (rd.sampler_x, rd.sampler_y, rd.n_dims, rd.jitter) == (7, 1, 0, 0)


@pytest.mark.parametrize("ns", [1, 2, 9])
def test_oracle_random_sampler_restatement_matches_the_mapping(ns):
    sc = O.OracleScene.readme(40, 24)
    rc, fr, _ = O.render(sc.desc, abi.render_desc(ns, 1, n_dims=0), threads=8, flags=ORACLE_FLAG_RANDOM_SAMPLER)
    rc2, fs, _ = O.render(sc.desc, random_desc(ns), threads=8)
    assert rc == rc2 == 0 and np.array_equal(fr.view(np.uint64), fs.view(np.uint64))
    if ns > 1:
        assert fr.max() > 0


def test_oracle_random_sampler_differs_from_stratified():
    sc = O.OracleScene.readme(40, 24)
    _, fr, _ = O.render(sc.desc, abi.render_desc(4, 1), threads=8, flags=ORACLE_FLAG_RANDOM_SAMPLER)
    _, fs, _ = O.render(sc.desc, abi.render_desc(4, 1), threads=8)
    assert not np.array_equal(fr, fs)


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", [abi.PBRT_INTEGRATOR_PATH, abi.PBRT_INTEGRATOR_DIRECT_LIGHTING])
@pytest.mark.parametrize("ns", [4, 16])
def test_device_random_sampler_vs_oracle(integrator, ns):
    scene = G.Scene.readme(64, 48)
    rd = random_desc(ns, integrator=integrator)
    rc, of, _ = O.render(scene.desc, abi.render_desc(ns, 1, n_dims=0, integrator=integrator), threads=8,
                         flags=ORACLE_FLAG_RANDOM_SAMPLER)
    assert rc == 0
    with G.Renderer(scene) as r:
        film, _ = r.render(rd)
    assert np.array_equal(film.view(np.uint64), of.view(np.uint64))
