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


def test_every_leg_has_a_fraction_and_kernel_traffic():
    c = bench.compact(_full())
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
    # the legs with a committed PMC summary carry their traffic
    for leg, sub in (("cfg4_sharded", None), ("spmv_unstructured", None), ("gmres", "spmv"), ("cfg5", "spmv"),
                     ("cfg5", "update"), ("gmres_metric", "mgs"), ("cfg2", None), ("spmv_general", None)):
        kr = legs[leg][sub] if sub else legs[leg]
        assert kr["traffic"] and kr["traffic"] > 0, (leg, sub)
        assert kr["traffic_src"].startswith("profiles/"), (leg, sub)
    assert c["roofline"]["traffic"] > 0


def test_traffic_requires_the_same_matrix():
    idx = bench.traffic_index()
    assert idx, "profiles/r05_traffic_index.json missing (tools/traffic_index.py)"
    e = idx["cfg4"]["spmv"]
    assert bench.leg_traffic(idx, "cfg4", "spmv", e["n"], e["nnz"])[0] == e["bytes"]
    assert bench.leg_traffic(idx, "cfg4", "spmv", e["n"] + 1, e["nnz"]) == (None, None)
