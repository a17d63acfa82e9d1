"""Multi-sequence serving loop over a paged batch.

The reference drives ONE sequence (iengine.cu:226-456; a second sequence is commented out
at iengine.cu:309-322, 369-373, 448-452) through ``llm()`` and grows a linked page list
per sequence (iengine.cu:73-109).  Here requests share the B slots of one ``Batch`` with
a paged KV cache: a waiting request is admitted into a free slot when the page pool can
hold its worst case (prompt + max_new_tokens), prefilled there while the other slots keep
decoding (requests admitted together with equal prompt lengths into consecutive slots
prefill in one ``qie_prefill_batch`` pass), and retired at its stop token / token budget, which returns its pages
(``qie_batch_release``).  Every step is one fixed-B decode step over all slots (idle
slots run on the scratch page and their outputs are dropped), so the hipGraph captured
for the batch is replayed unchanged.

One sampling configuration per batcher (``qie_sampling`` is per step); slot rows are
independent, so a request's tokens do not depend on what the other slots hold.
"""
from __future__ import annotations

import collections
import dataclasses
from typing import Deque, Dict, List, Optional, Sequence

from .engine import GREEDY, Batch, Engine, Sampling


@dataclasses.dataclass
class Request:
    rid: int
    prompt: List[int]
    max_new_tokens: int
    stop_ids: tuple = ()
    tokens: List[int] = dataclasses.field(default_factory=list)
    logits: list = dataclasses.field(default_factory=list)   # per token, when keep_logits
    slot: int = -1
    pages: int = 0
    done: bool = False


def prefill_runs(admitted: Sequence[Request]) -> List[List[Request]]:
    """Split requests (in admission order) into runs that one qie_prefill_batch call can
    take: consecutive slots, equal prompt lengths."""
    runs: List[List[Request]] = []
    for r in admitted:
        prev = runs[-1][-1] if runs else None
        if prev is not None and r.slot == prev.slot + 1 and len(r.prompt) == len(prev.prompt):
            runs[-1].append(r)
        else:
            runs.append([r])
    return runs


class ContinuousBatcher:
    def __init__(self, engine: Engine, slots: int = 8, max_ctx: Optional[int] = None, page_tokens: int = 128,
                 n_pages: int = 0, sampling: Sampling = GREEDY, keep_logits: bool = False):
        self.batch: Batch = engine.batch(slots, max_ctx, page_tokens=page_tokens, n_pages=n_pages)
        self.keep_logits = keep_logits          # copy each token's logit row (tests / diagnostics)
        self.max_ctx = self.batch.max_ctx
        self.sampling = sampling
        free, _, self.page_tokens = self.batch.page_stats()
        self.budget = free                      # pages not promised to an admitted request
        self.waiting: Deque[Request] = collections.deque()
        self.slots: List[Optional[Request]] = [None] * slots
        self.requests: Dict[int, Request] = {}
        self._next = 0

    def _pages(self, n_tokens: int) -> int:
        return -(-n_tokens // self.page_tokens)

    def submit(self, prompt: Sequence[int], max_new_tokens: int, stop_ids: Sequence[int] = ()) -> int:
        n = len(prompt)
        if n < 1 or max_new_tokens < 1 or n + max_new_tokens > self.max_ctx - 1:
            raise ValueError(f"request of {n} + {max_new_tokens} tokens does not fit max_ctx {self.max_ctx}")
        if self._pages(n + max_new_tokens) > self.budget + sum(r.pages for r in self.slots if r):
            raise ValueError("request larger than the whole page pool")
        r = Request(self._next, [int(t) for t in prompt], int(max_new_tokens), tuple(int(s) for s in stop_ids))
        self._next += 1
        self.requests[r.rid] = r
        self.waiting.append(r)
        return r.rid

    def _finish(self, r: Request) -> None:
        r.done = True
        self.batch.release(r.slot)
        self.slots[r.slot] = None
        self.budget += r.pages
        r.slot = -1

    def _emit(self, r: Request, tok: int, out: list, logits=None) -> None:
        r.tokens.append(tok)
        if self.keep_logits:
            r.logits.append((self.batch.logits() if logits is None else logits)[r.slot].copy())
        out.append((r.rid, tok))
        if len(r.tokens) >= r.max_new_tokens or tok in r.stop_ids:
            self._finish(r)

    def _admit(self, out: list) -> None:
        admitted: List[Request] = []
        while self.waiting:
            r = self.waiting[0]
            need = self._pages(len(r.prompt) + r.max_new_tokens)
            free_slot = next((i for i, s in enumerate(self.slots) if s is None), None)
            if free_slot is None or need > self.budget:
                break                           # FIFO: later requests wait behind the head
            self.waiting.popleft()
            r.slot, r.pages = free_slot, need
            self.budget -= need
            self.slots[free_slot] = r
            admitted.append(r)
        # equal-length prompts landing in consecutive slots prefill in one pass
        # (qie_prefill_batch); tokens are emitted in admission order afterwards
        first: Dict[int, int] = {}
        for run in prefill_runs(admitted):
            if len(run) == 1:
                first[run[0].rid] = self.batch.prefill(run[0].slot, run[0].prompt, self.sampling)
            else:
                toks = self.batch.prefill_batch(run[0].slot, [r.prompt for r in run], self.sampling)
                first.update((r.rid, t) for r, t in zip(run, toks))
        lg = self.batch.logits() if self.keep_logits and admitted else None
        for r in admitted:
            self._emit(r, first[r.rid], out, lg)

    def step(self) -> List[tuple]:
        """Admit what fits, then one decode step for every slot; returns the (request id,
        token) pairs produced, in slot order."""
        out: List[tuple] = []
        self._admit(out)
        if any(s is not None for s in self.slots):
            live = list(self.slots)
            ids = self.batch.decode_step(self.sampling)
            lg = self.batch.logits() if self.keep_logits else None
            for i, r in enumerate(live):
                if r is not None and not r.done:
                    self._emit(r, int(ids[i]), out, lg)
        return out

    def idle(self) -> bool:
        return not self.waiting and all(s is None for s in self.slots)

    def run(self) -> Dict[int, List[int]]:
        while not self.idle():
            self.step()
        return {rid: r.tokens for rid, r in self.requests.items()}

    def close(self) -> None:
        self.batch.close()
