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


def _bench(args, extra_env=None, timeout=600):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args + ["--no-cpu-baseline", "--no-latency"],
                          env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
@pytest.mark.parametrize("wl,batch", [("c4", 8), ("c5", 8), ("c5", 1)])
def test_bench_four_ranks_on_one_gpu(wl, batch):
    # rehearsal of the N-GPU path with 4 ranks (the ring wrap: rank 0 takes
    # rank 3's previous-step record); c5 at --batch 1 is configs[4]'s literal
    # shape, one frame pair in flight per rank.  Every rank's pipelined
    # matches must equal its serial loop's (bench.py aborts otherwise) and
    # the line must name all 4 ranks.
    r = _bench(["--gpus", "4", "--workload", wl, "--batch", str(batch), "--steps", "3", "--warmup", "1"],
               {"ORBX_BENCH_SHARE_GPU": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    dr = d["distributed"]
    assert d["n_gpus"] == 4 and dr["world_size"] == 4 and len(dr["ranks"]) == 4
    assert all(x["pipelined_equals_serial"] in (True, None) for x in dr["ranks"])
    assert all(x["matches_last_batch"] > 0 for x in dr["ranks"])


@pytest.mark.gpu
def test_bench_sharded_matches_equal_one_rank():
    # frame sharding changes who matches which pair, not the pairs: 4 ranks
    # x 2 frames match (0,7) (rank 0, across the ring wrap), (1,0), (2,1) ..
    # (7,6), the same pairs one rank x 8 frames matches, so the summed
    # keypoints and matches must be equal
    one = _bench(["--workload", "c1", "--batch", "8", "--steps", "2", "--warmup", "2"])
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = json.loads(one.stdout.strip().splitlines()[-1])
    four = _bench(["--gpus", "4", "--workload", "c1", "--batch", "2", "--steps", "2", "--warmup", "2"],
                  {"ORBX_BENCH_SHARE_GPU": "1"})
    assert four.returncode == 0, four.stderr[-3000:]
    d4 = json.loads(four.stdout.strip().splitlines()[-1])
    rk = d4["distributed"]["ranks"]
    assert sum(x["keypoints_last_batch"] for x in rk) == d1["config"]["keypoints_last_batch"]
    assert sum(x["matches_last_batch"] for x in rk) == d1["config"]["matches_last_batch"]


@pytest.mark.gpu
@pytest.mark.parametrize("fault", ["exit:1", "hang:1"])
def test_bench_failed_rank_ends_job(fault):
    # a rank that dies, or stops answering, must end the whole job non-zero
    # (no hang): launch_ranks stops the siblings of a failed rank, and a
    # parked rank trips the others' collective timeout
    import time
    t0 = time.time()
    r = _bench(["--gpus", "2", "--workload", "c1", "--batch", "4", "--steps", "2", "--warmup", "1"],
               {"ORBX_BENCH_SHARE_GPU": "1", "ORBX_BENCH_TEST_FAULT": fault, "ORBX_COLLECTIVE_TIMEOUT_S": "20"},
               timeout=300)
    assert r.returncode != 0
    assert "test fault" in r.stderr
    assert time.time() - t0 < 240
