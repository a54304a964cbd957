"""bench.py contract on CPU: the --gpus N launcher (torch.distributed.run as a
child, gloo stand-in step), the world-size guard, and the SURVEY §8(d) byte
attribution the roofline line uses."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--selftest-cpu", "--steps", "2", "--warmup", "1", "--config", "tsukuba",
              "--pairs-per-gpu", "3"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2
    assert d["config"]["global_batch"] == 6
    assert d["config"]["parallelism"] == "pairs/dp2"
    assert d["distributed"]["world_size"] == 2
    assert d["distributed"]["backend"] == "gloo"
    assert d["distributed"]["gathered_in_pair_order"] is True


def test_selftest_runs_mains_rank_path_three_ranks():
    # uneven shards of the same code path (3 ranks x 2 pairs), gathered in pair order
    r = _run(["--gpus", "3", "--selftest-cpu", "--steps", "2", "--warmup", "2", "--config", "tsukuba",
              "--pairs-per-gpu", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["distributed"]["world_size"] == 3
    # ranks 1, 2 send their blocks; rank 0 computed into its rows of the result
    assert d["distributed"]["gather_bytes_to_root"] == 4 * 288 * 384 * 2
    assert d["distributed"]["gathered_in_pair_order"] is True
    assert d["distributed"]["gather_exposed_ms_per_step"] >= 0


def test_selftest_four_ranks_overlapped_gather():
    # BASELINE config 4's shape at 4 ranks: double-buffered gather beside the next step
    r = _run(["--gpus", "4", "--selftest-cpu", "--steps", "3", "--warmup", "2", "--config", "tsukuba",
              "--pairs-per-gpu", "2"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    dd = d["distributed"]
    assert dd["world_size"] == 4 and dd["gathered_in_pair_order"] is True
    assert dd["gather_bytes_to_root"] == 6 * 288 * 384 * 2
    assert "double-buffered" in dd["gather"]


def test_dist_flag_one_rank():
    # --dist: the process group and the gather at world size 1 (what the GPU test runs over RCCL)
    r = _run(["--gpus", "1", "--dist", "--selftest-cpu", "--steps", "2", "--warmup", "1", "--config", "tsukuba"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1
    assert d["distributed"]["backend"] == "gloo" and d["distributed"]["world_size"] == 1
    assert d["distributed"]["gather_bytes_to_root"] == 0  # rank 0 computes into the result itself
    assert d["distributed"]["gathered_in_pair_order"] is True


def test_metric_names_the_config():
    assert bench.metric_for("kitti") == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert "Middlebury" in bench.metric_for("middlebury") and "2880×1988 D=256" in bench.metric_for("middlebury")
    assert "Tsukuba 384×288 D=16" in bench.metric_for("tsukuba")


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "2", "--selftest-cpu"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("mode,P", [("census8", 8), ("sgbm5", 5), ("sgbm8", 8), ("volume8", 8)])
@pytest.mark.parametrize("sweep", [False, True])
def test_stage_attribution_sums_to_model(mode, P, sweep):
    H, W, D = 375, 1242, 128
    stages = ("cost", "paths", "wta", "horizontal", "sweep", "sweep_wta", "median")
    tot = sum(bench.model_stage_bytes(s, mode, H, W, D, P, sweep) for s in stages)
    assert tot == bench.model_pair_bytes(mode, H, W, D, P)


def test_headline_model_numbers():
    # KITTI census 8 paths = 775.0 MB of volume traffic + I/O per pair
    H, W, D = 375, 1242, 128
    assert bench.model_pair_bytes("census8", H, W, D, 8) == 59_616_000 * 13 + 6 * H * W
    # per-direction aggregation owns P reads + the u16 S write: 10 B per cell (4.77 GB / 8 pairs)
    assert bench.model_stage_bytes("paths", "census8", H, W, D, 8, False) * 8 == 4_769_280_000


def test_kernel_stage_attribution_of_the_engines_kernels():
    """The PMC / SQ summaries sum a stage's kernels by name (tools/traffic_summary.py,
    valu_summary.py): the guarded fallback instances belong to no stage, the partial-only WTA
    instance (k_wta<..., false, true>) is the 5-path lines engine's WTA stage."""
    lines5 = ["void smk::k_sweep<16, 8, unsigned short, 3, 11>(smk::SweepArgs)",
              "void smk::k_ew_patch<16, 4, unsigned short>(smk::EwPatchArgs)",
              "void smk::k_wta<8, unsigned short, 1024, false, true>(smk::WtaArgs)",
              "void smk::k_wta<8, unsigned short, 1024, true, false>(smk::WtaArgs)",
              "void smk::k_sgm_paths<8, 16, 16, 8, false, unsigned short, true>(smk::PathsArgs)",
              "void smk::k_sgbm_cost2<2, 8, 1>(smk::SgbmCost2Args)"]
    st = {n: bench.kernel_stage(n, lines5) for n in lines5}
    assert st[lines5[0]] == "sweep" and st[lines5[1]] == "horizontal"
    assert st[lines5[2]] == "sweep_wta"
    assert st[lines5[3]] is None and st[lines5[4]] is None  # fallback instances
    assert st[lines5[5]] == "cost"
    lines8 = ["void smk::k_sweep<16, 8, unsigned char, 3, 11>(smk::SweepArgs)",
              "void smk::k_sweep<16, 8, unsigned char, 4, 11>(smk::SweepArgs)",
              "smk::k_lr_rows(unsigned int const*, unsigned int const*, short*, short*, int, int, int, int, int, int, int, unsigned int const*)"]
    assert [bench.kernel_stage(n, lines8) for n in lines8] == ["sweep", "sweep_wta", "wta"]
    perdir = ["void smk::k_sgm_paths<8, 16, 16, 8, true, unsigned char, false>(smk::PathsArgs)",
              "void smk::k_wta<8, unsigned char, 1024, false, false>(smk::WtaArgs)"]
    assert [bench.kernel_stage(n, perdir) for n in perdir] == ["paths", "wta"]
