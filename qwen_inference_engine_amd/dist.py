"""Minimal single-node process group for the multi-rank benchmark (no torch in-process).

One process per GPU, started by torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_PORT exported) or by bench.py's own launcher (which also exports QIE_GROUP_DIR, a
fresh directory).  Ranks only need a barrier, an all-gather of small JSON values (the RCCL
unique id) and a max over floats, so they meet through files.  The directory is unique to
the run: QIE_GROUP_DIR, else MASTER_PORT + the launcher's pid (all ranks of one
torch.distributed.run share their parent, the elastic agent) — files of an earlier run on
the same port can never satisfy a new barrier.  Rank 0 removes it at close().  Keeping
torch out of the process avoids loading a second HIP runtime beside libqie's (the wheel
bundles its own ROCm).
"""
from __future__ import annotations

import json
import os
import shutil
import time


def group_dir() -> str:
    d = os.environ.get("QIE_GROUP_DIR")
    if d:
        return d
    port = os.environ.get("MASTER_PORT", "0")
    run = os.environ.get("TORCHELASTIC_RUN_ID")
    if run:   # torch.distributed.run: the run id is shared by every rank (and unique to the run)
        return os.path.join("/tmp", f"qie_group_{port}_{run}")
    return os.path.join("/tmp", f"qie_group_{port}_{os.getppid()}")


class FileGroup:
    def __init__(self, rank: int, world: int, path: str = None, timeout: float = 300.0):
        self.rank, self.world = rank, world
        self.dir = path or group_dir()
        os.makedirs(self.dir, exist_ok=True)
        self.timeout = timeout
        self.gen = 0

    def _exchange(self, value):
        self.gen += 1
        path = os.path.join(self.dir, f"g{self.gen}_r{self.rank}.json")
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(value, f)
        os.replace(tmp, path)
        t0 = time.time()
        vals = [None] * self.world
        while True:
            done = True
            for r in range(self.world):
                if vals[r] is None:
                    p = os.path.join(self.dir, f"g{self.gen}_r{r}.json")
                    try:
                        with open(p) as f:
                            vals[r] = [json.load(f)]
                    except FileNotFoundError:
                        done = False
            if done:
                return [v[0] for v in vals]
            if time.time() - t0 > self.timeout:
                raise TimeoutError(f"rank {self.rank}: group exchange {self.gen} timed out in {self.dir}")
            time.sleep(0.0005)

    def barrier(self) -> None:
        self._exchange(0)

    def allgather(self, value):
        return self._exchange(value)

    def max(self, x: float) -> float:
        return max(self._exchange(float(x)))

    def close(self) -> None:
        """Final barrier; every rank then leaves a 'closed' marker (it reads nothing more),
        and rank 0 removes the rendezvous directory once all markers are there."""
        self.barrier()
        open(os.path.join(self.dir, f"closed_r{self.rank}"), "w").close()
        if self.rank == 0:
            t0 = time.time()
            while time.time() - t0 < self.timeout:
                if all(os.path.exists(os.path.join(self.dir, f"closed_r{r}")) for r in range(self.world)):
                    break
                time.sleep(0.001)
            shutil.rmtree(self.dir, ignore_errors=True)
