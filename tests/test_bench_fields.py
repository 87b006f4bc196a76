"""bench.py's roofline fields (host logic only): the bound the evidence names and the rocprof-based
fraction beside the event-based one."""
import bench


def test_bound_from_evidence():
    # cfg2 round 4: 34.4 MB per 47.5 us launch (0.09 of 8 TB/s), VALU issue 0.39 -> latency
    assert bench.roofline_bound(34.4e6, 47.5e-6, {"frac_valu_issue": 0.39})[0] == "latency"
    assert bench.roofline_bound(350e6, 47.5e-6, {"frac_valu_issue": 0.39})[0] == "hbm"
    assert bench.roofline_bound(34.4e6, 47.5e-6, {"frac_valu_issue": 0.8})[0] == "valu"
    # no PMC summary of this build: priced against HBM, no claim
    assert bench.roofline_bound(None, 47.5e-6, {"frac_valu_issue": None}) == ("hbm", None)


def test_rocprof_fraction():
    f = bench.rocprof_fields({"rocprof_avg_ns": 45680.0}, 16.05e6)
    assert f["rocprof_avg_launch_us"] == 45.68
    assert abs(f["frac_rocprof"] - 16.05e6 / 45.68e-6 / 8e12) < 1e-5
    assert bench.rocprof_fields({}, 1.0) == {"rocprof_avg_launch_us": None, "frac_rocprof": None}


def test_shard_choice_explained(monkeypatch):
    # config.parallelism says why the ranks run their decomposition: the measured sums, the
    # environment's request, or the shape's only option
    class E:
        shard_info = {"t_gather": 51.4, "t_partials": 42.7, "l_allreduce": 20.0, "l_allgather_state": 22.0,
                      "l_allgather_partials": 21.0}
    why = bench.shard_why(E())
    assert "gather 51.4 + all-gather 22.0 = 73.4 us" in why and "= 104.7 us" in why
    E.shard_info = None
    monkeypatch.delenv("STOMP_SHARD_MODE", raising=False)
    assert "only decomposition" in bench.shard_why(E())
    monkeypatch.setenv("STOMP_SHARD_MODE", "partials")
    assert "STOMP_SHARD_MODE" in bench.shard_why(E())
