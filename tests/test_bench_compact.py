"""bench.py's compact line (host logic, no device): the driver keeps only an
~8 KB tail of stdout, so the printed line must stay <= 6 KB and still carry
every leg's rate, dominant kernel, bytes per launch, frac and traffic."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGS = ("cfg4_sharded", "spmv_general", "spmv_unstructured", "gmres", "gmres_metric", "gmres_metric_restarted",
        "bicgstab_cfg3", "end_to_end", "cfg2", "cfg5")


def _full():
    # a verbose line of round 4 (profiles/r04_final_bench.json), with the n / nnz
    # the SpMV legs carry since round 5
    with open(os.path.join(REPO, "profiles", "r04_final_bench.json")) as f:
        full = json.load(f)
    for leg in ("spmv_general", "spmv_unstructured"):
        full[leg].update(n=10_077_696, nnz=149_770_936)
    return full


def test_compact_line_fits_the_driver_tail():
    c = bench.compact(_full())
    line = json.dumps(c)
    assert len(line) <= 6144
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in c, k
    assert set(LEGS) <= set(c["legs"])
    assert c["formulas"] == bench.FORMULAS and os.path.exists(os.path.join(REPO, bench.FORMULAS))


def _index(build):
    """An index of every leg's traffic taken on `build` (the committed one's
    layout, tools/traffic_index.py)."""
    e = lambda n, nnz: {"n": n, "nnz": nnz, "bytes": 1.0e9, "src": "profiles/r06_pmc_legs/x.json",  # noqa: E731
                        "build": build}
    M, C3, C4, C5, C2 = (10_077_696, 149_770_936), (2_000_000, 39_999_788), (10_004_569, 50_010_193), \
        (8_000_000, 55_760_000), (1_000_000, 4_996_000)
    return {"build": build, "metric_cg": {"spmv": e(*M)}, "spmv_general": {"spmv": e(*M)},
            "spmv_unstructured": {"spmv": e(*M)}, "gmres": {"spmv": e(*C3), "mgs": e(*C3)},
            "bicgstab_cfg3": {"spmv": e(*C3)}, "gmres_metric": {"spmv": e(*M), "mgs": e(*M)},
            "cfg4": {"spmv": e(*C4)}, "cfg5": {"spmv": e(*C5), "update": e(*C5)}, "cfg2": {"iteration": e(*C2)}}


def test_every_leg_has_a_fraction_and_kernel_traffic():
    from krylov_amd import _lib

    c = bench.compact(_full(), idx=_index(_lib.build_id()))
    legs = c["legs"]

    def kernels(leg):
        v = legs[leg]
        subs = [v[k] for k in ("spmv", "mgs", "update") if isinstance(v.get(k), dict)]
        return subs or [v]

    for leg in LEGS:
        if leg in ("gmres_metric_restarted", "end_to_end"):
            continue  # call-level rates, no single kernel
        for kr in kernels(leg):
            assert isinstance(kr["frac"], float) and 0.0 < kr["frac"] < 1.5, (leg, kr)
            assert kr["kernel"] and "<" not in kr["kernel"], (leg, kr)
    # every leg's traffic from an index taken on the loaded build
    for leg, sub in (("cfg4_sharded", None), ("spmv_unstructured", None), ("gmres", "spmv"), ("gmres", "mgs"),
                     ("cfg5", "spmv"), ("cfg5", "update"), ("gmres_metric", "mgs"), ("cfg2", None),
                     ("spmv_general", None), ("bicgstab_cfg3", None)):
        kr = legs[leg][sub] if sub else legs[leg]
        assert kr["traffic"] and kr["traffic"] > 0, (leg, sub)
        assert kr["traffic_src"].startswith("profiles/"), (leg, sub)


def test_traffic_of_another_build_is_null():
    """A PMC summary of other code is not evidence for this one: an index
    stamped with another build gives traffic: null on every leg."""
    c = bench.compact(_full(), idx=_index("0000000000000000"))
    legs = c["legs"]
    for leg in ("cfg4_sharded", "spmv_unstructured", "cfg2", "spmv_general", "bicgstab_cfg3"):
        assert legs[leg]["traffic"] is None, leg
    assert legs["gmres"]["mgs"]["traffic"] is None and legs["cfg5"]["update"]["traffic"] is None


def test_traffic_requires_the_same_matrix_and_build():
    from krylov_amd import _lib

    idx = _index(_lib.build_id())
    e = idx["cfg4"]["spmv"]
    assert bench.leg_traffic(idx, "cfg4", "spmv", e["n"], e["nnz"])[0] == e["bytes"]
    assert bench.leg_traffic(idx, "cfg4", "spmv", e["n"] + 1, e["nnz"]) == (None, None)
    assert bench.leg_traffic(_index("f" * 16), "cfg4", "spmv", e["n"], e["nnz"]) == (None, None)


def test_committed_traffic_index_is_of_the_shipped_library():
    """profiles/r06_traffic_index.json was taken on the library in the tree
    (its stamp is this build's), so the bench line's traffic figures describe
    the code that runs."""
    from krylov_amd import _lib

    if _lib.HOST_ONLY:
        import pytest

        pytest.skip("host-only build")
    idx = bench.traffic_index()
    assert idx, "profiles/r06_traffic_index.json missing (tools/pmc_legs.sh, tools/traffic_index.py)"
    assert idx["build"] == _lib.build_id(), "traffic index stamped with another build: re-take the PMC passes"
    for leg, ks in idx.items():
        if leg != "build":
            assert all(v["build"] == idx["build"] for v in ks.values()), leg


def test_traffic_index_covers_every_leg_kernel():
    """Every (leg, kernel) tools/traffic_index.py names resolves in the
    committed PMC summaries, so no leg prints traffic: null for a kernel-name
    mismatch (round 6: anonymous-namespace kernels were missed by a
    'void kry::' prefix)."""
    import importlib.util
    import os

    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("traffic_index", os.path.join(here, "tools", "traffic_index.py"))
    ti = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ti)
    idx = bench.traffic_index()
    for leg, (_fname, _shape, keys) in ti.LEGS.items():
        for key in keys:
            assert key in idx.get(leg, {}), (leg, key)
    assert "iteration" in idx["cfg2"]
