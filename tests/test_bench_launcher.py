"""bench.py's multi-GPU entry point on CPU (no GPU touched): `--gpus N` without a launcher
spawns N rank processes itself and reports n_gpus = N; under torch.distributed.run a
WORLD_SIZE that disagrees with --gpus is refused instead of mislabelling the run; the synthetic
corpus is distinct per block and deterministic."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def _line(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_ranks(n):
    r = _run(["--gpus", str(n), "--selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == n and d["ranks_reporting"] == n
    assert d["blocks_total"] == 4096 * n and d["scaling"] == "weak"


def test_config5_strong_split():
    r = _run(["--gpus", "2", "--total-blocks", "1048576", "--selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["blocks_total"] == 1048576 and d["scaling"] == "strong"


def test_dead_rank_does_not_hang_the_launcher():
    # rank 1 exits before the first collective: the launcher must kill rank 0 (blocked in gloo)
    # and report rank 1's status instead of waiting for gloo's 30-minute timeout
    r = _run(["--gpus", "2", "--selftest"], {"S3HC_SELFTEST_FAIL_RANK": "1"}, timeout=120)
    assert r.returncode == 3


def test_mismatched_world_size_is_refused():
    r = _run(["--gpus", "8", "--selftest"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_single_gpu_default_needs_no_launcher():
    r = _run(["--selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert _line(r.stdout)["n_gpus"] == 1


def test_synthetic_corpus_distinct_and_deterministic():
    import synth

    d = synth.log_text(256 * 65536, 123)
    assert d == synth.log_text(256 * 65536, 123, threads=1)
    assert d != synth.log_text(256 * 65536, 124)
    assert len({hashlib.sha1(d[i:i + 65536]).digest() for i in range(0, len(d), 65536)}) == 256
    assert synth.log_text(1000, 5) == synth.log_text(5000, 5)[:1000]  # prefix-stable
    j = synth.json_records(64 * 65536, 7)
    assert j.startswith(b'{"id":1,') and len({j[i:i + 65536] for i in range(0, len(j), 65536)}) == 64
    m, modes = synth.mixed_blocks(6, 65536)
    assert modes == [0, 1, 0, 1, 0, 1] and m[65536:65540] == b"\xff\xd8\xff\xe0"


def test_assign_device_refuses_shared_gpus():
    # one process per GPU: N ranks on fewer than N visible devices must not report N GPUs
    sys.path.insert(0, ROOT)
    import bench

    assert bench.assign_device(8, 3, 8, False) == (3, None)
    assert bench.assign_device(1, 0, 1, False) == (0, None)
    dev, why = bench.assign_device(8, 3, 1, False)
    assert dev is None and "refusing" in why and "--share-gpu" in why
    assert bench.assign_device(8, 3, 1, True) == (0, None)  # explicit rehearsal
    assert bench.assign_device(2, 1, 4, True) == (1, None)
    assert bench.assign_device(1, 0, 0, True)[0] is None    # no device at all
    dev, why = bench.assign_device(2, 2, 2, False)          # a local rank past the devices
    assert dev is None and "LOCAL_RANK" in why


def test_gpus_flag_refused_without_enough_devices():
    # this container has no GPU: two ranks are refused before any collective or HIP work,
    # and the launcher reports the refusal's status instead of a bench line
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "visible GPU" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
