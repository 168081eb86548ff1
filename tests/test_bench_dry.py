"""bench.py's multi-GPU control flow on CPU (--dry-run-cpu: gloo + a stub engine
that computes no pairing): `--gpus N` without a launcher starts N ranks itself,
shards config 4's rows contiguously, all-gathers every chunk inside the step,
takes the max time over ranks and cross-checks a sample of the next rank's
rows.  The GPU path of the same code runs in the driver's N-GPU bench."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=e, cwd=ROOT)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_spawns_ranks_config4(world):
    r = run(["--gpus", str(world), "--dry-run-cpu", "--steps", "1", "--warmup", "1", "--total", "16384",
             "--chunk", "2048"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["dry_run"] is True
    assert line["config"]["workload"].startswith("BASELINE config 4")
    assert line["config"]["total_pairs"] == 16384 and line["config"]["pairs_per_gpu"] == 16384 // world
    assert line["scaling"] == "strong" and line["config"]["allgather_in_step"]
    assert line["cross_rank_check"]["mismatches"] == 0 and line["cross_rank_check"]["ranks_ok"] == world
    # rank 0's checker leg over the gathered rows: 4096 rows spread over every shard
    sc = line["sample_check"]
    assert sc["rows"] == 4096 and sc["mismatches"] == 0 and sc["parity_sample_bit_exact"] is True
    assert sc["first_row"] == 0 and sc["last_row"] == 16383
    cb = line["cpu_baseline"]
    assert cb["parity_sample_bit_exact"] is True and cb["value"] > 0 and cb["kind"] == "dry-run stub"
    assert {"cores", "single_core", "cpu_model", "sample", "unit"} <= set(cb)
    assert line["collective"]["world_from_allreduce"] == world


def test_sample_blocks_cover_every_shard():
    sys.path.insert(0, ROOT)
    import bench
    total = 1 << 20
    blocks = bench.sample_blocks(total)
    assert sum(b - a for a, b in blocks) == 4096 and blocks[0][0] == 0 and blocks[-1][1] == total
    for world in (2, 4, 8):
        per = total // world
        assert {a // per for a, _ in blocks} == set(range(world))
    assert bench.sample_blocks(100) == [(0, 100)]


def test_bench_world_size_must_match_gpus():
    r = run(["--gpus", "2", "--dry-run-cpu"], env={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


@pytest.mark.parametrize("ndev", [1, 3, 8])
def test_bench_capi_form_keys(ndev):
    """`--form capi`: config 4 in one process over N devices (bn_ctx_create_multi +
    bn_pairing_many_allgather_dev on the GPU); here the stub engine: no ranks are
    spawned, every device's gathered buffer is compared with device 0's, and rank
    0's checker sample and cpu_baseline keys are the torch form's."""
    r = run(["--gpus", str(ndev), "--form", "capi", "--dry-run-cpu", "--steps", "2", "--warmup", "1",
             "--total", "12288"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "launching" not in r.stderr  # no torch.distributed.run child
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == ndev and line["dry_run"] is True and line["steps"] == 2
    assert line["config"]["form"] == "capi" and line["config"]["total_pairs"] == 12288
    assert line["config"]["pairs_per_gpu"] == 12288 // ndev and line["scaling"] == "strong"
    assert line["collective"]["devices_equal_to_device0"] is True and line["collective"]["world_from_allreduce"] == ndev
    sc = line["sample_check"]
    assert sc["mismatches"] == 0 and sc["parity_sample_bit_exact"] is True and sc["last_row"] == 12287
    assert line["cpu_baseline"]["kind"] == "dry-run stub" and line["value"] > 0


def test_bench_capi_form_rejects_launcher_and_workloads():
    r = run(["--gpus", "2", "--form", "capi", "--dry-run-cpu"], env={"WORLD_SIZE": "2", "RANK": "0",
                                                                    "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--form capi" in r.stderr
    r = run(["--form", "capi", "--workload", "g1mul", "--dry-run-cpu"])
    assert r.returncode == 2
    r = run(["--workload", "g2mul", "--gpus", "2", "--dry-run-cpu"], env={"WORLD_SIZE": "2", "RANK": "0",
                                                                      "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "runs on one GPU" in r.stderr


def test_bench_under_the_drivers_launcher_world8():
    """The driver's own N = 8 command line (torch.distributed.run with eight ranks on
    127.0.0.1, bench.py --gpus 8 in every rank), with the stub engine on gloo: the
    exact control flow of SCALE's 8-GPU point."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "8", "--steps", "1", "--warmup", "1", "--dry-run-cpu", "--total", "16384",
                        "--chunk", "2048"], capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints the line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8 and line["config"]["pairs_per_gpu"] == 2048
    assert line["cross_rank_check"]["ranks_ok"] == 8 and line["collective"]["world_from_allreduce"] == 8
    assert line["sample_check"]["mismatches"] == 0
