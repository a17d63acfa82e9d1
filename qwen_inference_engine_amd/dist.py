"""Minimal single-node process group for replica benchmarks (no torch in-process).

torch.distributed.run launches one process per GPU and exports RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_PORT.  Replica ranks only need a barrier and a max/sum over a few
floats, so they meet through files under /tmp keyed by MASTER_PORT (all ranks share
one node).  Keeping torch out of the process avoids loading a second HIP runtime
beside libqie's (the wheel bundles its own ROCm).
"""
from __future__ import annotations

import json
import os
import time


class FileGroup:
    def __init__(self, rank: int, world: int, tag: str = None, timeout: float = 600.0):
        self.rank, self.world = rank, world
        tag = tag or os.environ.get("MASTER_PORT", "0")
        self.dir = os.path.join("/tmp", f"qie_group_{tag}_{os.environ.get('TORCHELASTIC_RUN_ID', 'x')}")
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
                    if os.path.exists(p):
                        with open(p) as f:
                            vals[r] = json.load(f)
                    else:
                        done = False
            if done:
                return vals
            if time.time() - t0 > self.timeout:
                raise TimeoutError(f"rank {self.rank}: group exchange {self.gen} timed out")
            time.sleep(0.0005)

    def barrier(self) -> None:
        self._exchange(0)

    def allgather(self, value):
        return self._exchange(value)

    def max(self, x: float) -> float:
        return max(self._exchange(float(x)))
