"""bench.py's roofline pricing (CPU): the bound it names is the path that ran, and `frac` is a
fraction of a ceiling that path can reach (<= 1 at the measured C2/C3/C4 rates)."""
import bench


class _Ctx:
    def __init__(self, brute):
        self.brute = brute

    def scene_info(self):
        return {"brute_records": 36 if self.brute else 0, "brute_boxes": 22 if self.brute else 0,
                "nodes": 7255, "tris": 7256}

    def work_bytes(self):
        return {"box_test": 32.0, "tri_test": 36.0, "ray": 40.0, "env_lookup": 16.0}


def _counts(per_sample, samples):
    keys = list(bench.VALU_OPS) + ["node_fetches"]
    c = {k: 0 for k in keys}
    c.update({k: v * samples for k, v in per_sample.items()})
    c["samples"] = samples
    return c


def test_brute_force_priced_on_valu():
    # C2 per-sample counts of BENCH r02 (brute force), 7.92 ms per 1024^2 x 64 frame
    s = 1024 * 1024 * 64
    cnt = _counts({"box_tests": 78.78, "tri_tests": 14.24, "rays": 3.58, "ev_diffuse": 2.99, "sun_terms": 0.6,
                   "node_fetches": 34.6}, s)
    rf = bench.roofline(_Ctx(True), cnt, 7.92, 1024 * 1024, "no_such_workload")
    assert rf["bound"] == "valu" and rf["unit"] == "Tops/s"
    assert 0.2 < rf["frac"] <= 1.0
    assert "survey_bytes_model" in rf   # the byte model is reported, never as an HBM fraction


def test_tree_walk_priced_on_cache_not_hbm():
    # C4: 1920x1080 x 512 spp in 450.6 ms; its SURVEY 8(d) bytes exceed 8 TB/s (served by vL1D / L2)
    s = 1920 * 1080 * 512
    cnt = _counts({"box_tests": 95.0, "tri_tests": 18.2, "rays": 0.97, "node_fetches": 95.0 / 2,
                   "env_lookups": 1.0}, s)
    rf = bench.roofline(_Ctx(False), cnt, 450.6, 1920 * 1080, "no_such_workload")
    assert rf["bound"] == "cache" and rf["peak"] == bench.CACHE_PEAK_GBS
    assert rf["achieved"] > bench.HBM_PEAK_GBS * 0.5   # the byte rate an HBM fraction would have mispriced
    assert 0.0 < rf["frac"] <= 1.0
    assert rf["hbm_measured"]["peak"] == bench.HBM_PEAK_GBS
