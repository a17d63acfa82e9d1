"""CPU: bench.py's multi-GPU launcher and the rank rendezvous, without any GPU.

* `bench.py --gpus N --dry-run` (no WORLD_SIZE) stops before libqie loads and prints the
  environment of each of the N child ranks it would start: RANK / LOCAL_RANK 0..N-1, one
  WORLD_SIZE, one MASTER_PORT on 127.0.0.1 and one fresh rendezvous directory.
* FileGroup (qwen_inference_engine_amd.dist): barrier / all-gather / max across real
  processes; the directory is unique per run and removed at close, so files of an earlier
  run cannot satisfy a new barrier.
* tp_shardable: which BASELINE models run tensor-parallel at 2 / 4 / 8 GPUs.
"""
import json
import multiprocessing as mp
import os
import subprocess
import sys

from conftest import ROOT

from qwen_inference_engine_amd import spec as S
from qwen_inference_engine_amd.dist import FileGroup


def test_launcher_dry_run_child_environments():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "QIE_GROUP_DIR")}
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                                  env=env, timeout=120).decode()
    kids = json.loads(out.strip().splitlines()[-1])
    assert [k["RANK"] for k in kids] == ["0", "1", "2", "3"]
    assert [k["LOCAL_RANK"] for k in kids] == ["0", "1", "2", "3"]
    assert {k["WORLD_SIZE"] for k in kids} == {"4"}
    assert {k["MASTER_ADDR"] for k in kids} == {"127.0.0.1"}
    assert len({k["MASTER_PORT"] for k in kids}) == 1 and len({k["QIE_GROUP_DIR"] for k in kids}) == 1
    assert os.path.isdir(kids[0]["QIE_GROUP_DIR"])
    os.rmdir(kids[0]["QIE_GROUP_DIR"])


def test_launcher_respects_torchrun_world():
    """Under torch.distributed.run (WORLD_SIZE set) bench.py is a rank, not a launcher."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    out = subprocess.check_output([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                                  env=env, timeout=120).decode()
    assert json.loads(out.strip().splitlines()[-1]) == {"world": 2}


def _member(rank, world, path, q):
    g = FileGroup(rank, world, path=path, timeout=60)
    g.barrier()
    got = g.allgather({"r": rank})
    mx = g.max(float(rank) * 1.5)
    g.close()
    q.put((rank, got, mx))


def test_file_group_three_processes(tmp_path):
    path = str(tmp_path / "grp")
    # stale files of an earlier run in an OLD directory are never read: each run gets its own
    os.makedirs(str(tmp_path / "old"), exist_ok=True)
    open(str(tmp_path / "old" / "g1_r0.json"), "w").write("0")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_member, args=(r, 3, path, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r, got, mx in res:
        assert got == [{"r": 0}, {"r": 1}, {"r": 2}]
        assert mx == 3.0
    assert not os.path.exists(path)          # rank 0 removed the rendezvous directory


def test_tp_shardable_presets():
    ok = {(n, tp): S.tp_shardable(S.PRESETS[n], tp)[0] for n in S.PRESETS for tp in (2, 4, 8)}
    assert ok[("Qwen2-7B", 2)] and ok[("Qwen2-7B", 4)] and ok[("Qwen2-7B", 8)]   # 8: kv heads replicated
    assert ok[("Qwen2-72B", 8)] and ok[("Qwen3-14B", 8)]
    assert [S.shard_heads(28, 4, 8, r)[0] for r in range(8)] == [4, 3, 4, 3, 4, 3, 4, 3]
    assert S.shard_heads(28, 4, 32, 0) is None       # 8 ranks per kv head > its 7 q heads
    assert S.shard_heads(28, 4, 6, 0) is None        # 6 neither divides nor is a multiple of 4


def test_pmc_traffic_is_read_from_the_benched_configuration():
    """bench.py's roofline.traffic comes from the PMC summary of the configuration it ran:
    the headline (bf16, B = 1) never picks up config 4's (fp8, B = 8) file and vice versa."""
    sys.path.insert(0, ROOT)
    import bench
    head, src = bench.pmc_traffic("gate_up", "")
    assert src is not None and "fp8" not in src and head > 2.5e8   # 271.6 MB algorithmic
    fp8, src8 = bench.pmc_traffic("gate_up", "fp8_b8_")
    assert src8 is not None and "fp8_b8" in src8 and 1.3e8 < fp8 < 1.5e8   # 136.2 MB algorithmic
