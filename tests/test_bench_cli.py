"""bench.py contract checks that need no GPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_beyond_visible_devices_fails_loudly():
    # --gpus N without WORLD_SIZE starts N ranks; with fewer GPUs visible it
    # must exit non-zero before touching any device (no silent 1-GPU run)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""  # none visible, also on a GPU box
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_bench_byte_models():
    sys.path.insert(0, ROOT)
    import bench
    import orbx
    geo = orbx.geometry(orbx.params(2000, 1.2, 8, 20, 7, "empty"), 1920, 1080)
    by = bench.stage_bytes(geo, 1, 0, 0, 2000)
    # B_pyr+FAST at 1080p / 8 levels counts level 1 (= level 0,
    # partial_sum quirk) as its own level; orbx aliases it, so FAST reads and
    # resize moves only the unique levels
    P = [w * h for w, h in zip(geo.level("width"), geo.level("height"))]
    assert by["fast_cells"] == sum(P) - P[1]
    assert bench.min_pyr_fast_bytes(geo, 1) == sum(P) - P[1]


import json  # noqa: E402

import pytest  # noqa: E402


@pytest.mark.gpu
def test_bench_pipelined_step_runs_and_matches_serial():
    # the default bench line times the pipelined step (extraction of step
    # k+1 overlapping the matching of step k); bench.py itself aborts if its
    # matches differ from the serial loop's, and reports the serial numbers
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c1", "--batch", "8",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-latency"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["serial"]["value"] > 0 and "pipelined" in d["step_mode"]
    assert d["config"]["matches_last_batch"] > 0


@pytest.mark.gpu
def test_bench_split_extraction_matches_serial():
    # --split 2: the pipelined step extracts the batch as two sub-batches on
    # two streams (two plans); bench.py aborts unless the matches equal the
    # serial loop's (one plan over the whole batch)
    # (c5: left + right plans and a stereo plan per sub-batch)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    for wl in ("c1", "c5"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", wl, "--batch", "8",
                            "--split", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-latency"],
                           env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["value"] > 0 and "2 sub-batches" in d["step_mode"]


@pytest.mark.gpu
def test_bench_two_ranks_pipelined_on_one_gpu():
    # rehearsal of the N-GPU bench path on one GPU (both ranks on cuda:0,
    # boundary exchange over gloo): the serial loop runs the ring exchange,
    # the pipelined loop runs it on the extraction stream, and bench.py
    # aborts unless both give the same matches on every rank
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ORBX_BENCH_SHARE_GPU"] = "1"
    for wl in ("c1", "c5"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", wl,
                            "--batch", "8", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-latency"],
                           env=env, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["n_gpus"] == 2 and d["value"] > 0 and d["serial"]["value"] > 0


@pytest.mark.gpu
def test_bench_c4_host_fed_and_latency_legs():
    # the c4 line's extra legs at a small batch: frames fed from pinned host
    # memory over two copy streams must give the resident run's keypoint
    # counts with every keypoint row returned; the drop-in latency leg (C ABI
    # and the reference-shaped compat operator()) reports every call site
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c4", "--batch", "8",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    hf = d["host_fed"]
    assert hf["value"] > 0 and hf["counts_equal_resident_run"] and hf["rows_cover_all_keypoints"]
    assert hf["h2d_streams"] == 2
    lat = d["latency"]
    for k in ("extract_640x480", "extract_1920x1080", "search_by_bow_2000x2000"):
        assert lat[k]["p50_us"] > 0 and lat[k]["p99_us"] >= lat[k]["p50_us"]
    co = lat["compat_operator_1920x1080"]
    assert co["operator_with_mvImagePyramid"]["checksum"] != 0
    assert co["operator_with_mvImagePyramid"]["keypoints"] == co["operator_no_pyramid"]["keypoints"]
