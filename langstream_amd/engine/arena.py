"""Step arena: the fixed binary layout in which the scheduler describes one engine step.

The Python scheduler fills a pinned host arena through numpy views (no torch calls,
so no GIL hand-offs), and the native ``StepExecutor`` (``ops/csrc/runner.hip``) runs
the whole step from it in one GIL-released call: one H2D copy, token feedback,
forward, logit deltas, sampling, one D2H copy.  Under tensor parallelism the device
copy of the arena is what rank 0 broadcasts to the other ranks.

``PyStepExecutor`` runs the same arena on the CPU (model.forward_logits + reference
sampling) so the scheduler has ONE code path, exercised by the CPU test-suite.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..models.llama import AttnMeta

# header words (must match enum Hdr in runner.hip)
H_KIND, H_T, H_ND, H_NPS, H_NTILES, H_NROWS, H_NGATHER, H_NDELTA, H_NTOP, H_BUCKET, H_ROWS_ALL, H_NCOPY = range(12)
KIND_STEP, KIND_STOP, KIND_CAPTURE = 1, 3, 4
MAX_KV_COPIES = 2048   # KV block copies a step can carry (kMaxKvCopies in runner.hip)
MAX_TOP = 32
_ALIGN = 256


@dataclass
class ArenaLayout:
    max_tokens: int
    max_seqs: int
    max_blocks: int
    max_tiles: int
    max_deltas: int
    offsets: Dict[str, int]
    fields: Dict[str, Tuple[np.dtype, tuple]]
    fixed_bytes: int
    nbytes: int

    @staticmethod
    def build(max_tokens: int, max_seqs: int, max_blocks: int, max_tiles: int, max_deltas: int) -> "ArenaLayout":
        T, S, B = max_tokens, max_seqs, max_blocks
        spec = [("hdr", np.int32, (16,)), ("ids", np.int32, (T,)), ("pos", np.int32, (T,)),
                ("slots", np.int64, (T,)), ("dbt", np.int32, (S, B)), ("dctx", np.int32, (S,)),
                ("pbt", np.int32, (S, B)), ("q_start", np.int32, (S,)), ("q_len", np.int32, (S,)),
                ("ctx_len", np.int32, (S,)), ("tiles", np.int32, (max_tiles, 2)), ("rows", np.int64, (S,)),
                ("gdst", np.int64, (S,)), ("gsrc", np.int64, (S,)), ("temp", np.float32, (S,)),
                ("top_p", np.float32, (S,)), ("top_k", np.int32, (S,)), ("seeds", np.int64, (S,)),
                ("steps", np.int64, (S,)), ("kvcopy", np.int32, (MAX_KV_COPIES, 2)),
                ("deltas", np.int32, (max_deltas, 3))]
        off, fields, cur = {}, {}, 0
        for name, dt, shape in spec:
            cur = (cur + _ALIGN - 1) // _ALIGN * _ALIGN
            off[name] = cur
            fields[name] = (np.dtype(dt), shape)
            if name == "deltas":
                fixed = cur
            cur += int(np.prod(shape)) * np.dtype(dt).itemsize
        return ArenaLayout(T, S, B, max_tiles, max_deltas, off, fields, fixed, cur)

    def views(self, buf: np.ndarray) -> Dict[str, np.ndarray]:
        assert buf.dtype == np.uint8 and buf.size >= self.nbytes
        out = {}
        for name, (dt, shape) in self.fields.items():
            o = self.offsets[name]
            n = int(np.prod(shape)) * dt.itemsize
            out[name] = buf[o: o + n].view(dt).reshape(shape)
        return out


def out_views(buf: np.ndarray, max_seqs: int) -> Dict[str, np.ndarray]:
    S = max_seqs
    return {"tok": buf[0: 4 * S].view(np.int32), "lp": buf[4 * S: 8 * S].view(np.float32),
            "ti": buf[8 * S: 8 * S + 4 * S * MAX_TOP].view(np.int32),
            "tl": buf[8 * S + 4 * S * MAX_TOP: 8 * S + 8 * S * MAX_TOP].view(np.float32)}


def out_bytes(max_seqs: int) -> int:
    return max_seqs * 8 + max_seqs * MAX_TOP * 8


class NativeStepExecutor:
    """Thin holder for the C++ executor plus numpy views of its pinned slots."""

    def __init__(self, model, kv_caches, layout: ArenaLayout, nslots: int, nsplit: int, bps: int,
                 use_graphs: bool, device: torch.device):
        runner = model._native_runner(kv_caches)
        self.layout = layout
        self.x = ops.hip().StepExecutor(runner, dict(layout.offsets), layout.nbytes, layout.fixed_bytes,
                                        layout.max_tokens, layout.max_seqs, layout.max_blocks, layout.max_tiles,
                                        layout.max_deltas, nslots, nsplit, bps, use_graphs,
                                        device.index if device.index is not None else torch.cuda.current_device())
        self.inputs = [layout.views(self.x.host_slot(i).numpy()) for i in range(nslots)]
        self.outputs = [out_views(self.x.out_slot(i).numpy(), layout.max_seqs) for i in range(nslots)]
        self.wait_in = self.x.wait_in
        self.wait_out = self.x.wait_out
        self.launch = self.x.launch
        self.step = self.x.step
        self.timings = self.x.timings
        self.capture = self.x.capture
        self.has_graph = self.x.has_graph
        self.shutdown = self.x.shutdown
        self.worker_loop = self.x.worker_loop


class PyStepExecutor:
    """CPU (or debugging) executor with the native executor's semantics."""

    def __init__(self, model, kv_caches, layout: ArenaLayout, nslots: int, nsplit: int, bps: int,
                 device: torch.device, tp_group=None, tp_world: int = 1):
        self.model = model
        self.kv = kv_caches
        self.layout = layout
        self.nsplit, self.bps = nsplit, bps
        self.device = device
        self.tp_group, self.tp_world = tp_group, tp_world
        self._in = [np.zeros(layout.nbytes, np.uint8) for _ in range(nslots)]
        self._out = [np.zeros(out_bytes(layout.max_seqs), np.uint8) for _ in range(nslots)]
        self.inputs = [layout.views(b) for b in self._in]
        self.outputs = [out_views(b, layout.max_seqs) for b in self._out]
        self._arena = np.zeros(layout.nbytes, np.uint8)
        self._av = layout.views(self._arena)
        self._tok = np.zeros(layout.max_seqs, np.int32)
        self._graphs = set()
        self._ws = torch.empty(max(1, layout.max_seqs * model.hq * nsplit * (model.cfg.head_dim + 2)),
                               dtype=torch.float32, device=device)

    def wait_in(self, i: int) -> None:
        pass

    def wait_out(self, i: int) -> None:
        pass

    def has_graph(self, B: int) -> bool:
        return B in self._graphs

    def capture(self, B: int) -> None:
        if self.tp_world > 1:
            self._announce(KIND_CAPTURE, B)
        self._graphs.add(B)

    def shutdown(self) -> None:
        if self.tp_world > 1:
            self._announce(KIND_STOP, 0)

    def _announce(self, kind: int, B: int) -> None:
        self._av["hdr"][:] = 0
        self._av["hdr"][H_KIND] = kind
        self._av["hdr"][H_BUCKET] = B
        self._bcast()

    def _bcast(self) -> None:
        t = torch.from_numpy(self._arena)
        dist.broadcast(t, src=dist.get_global_rank(self.tp_group, 0) if self.tp_group is not None else 0,
                       group=self.tp_group)

    def step(self, slot: int, prev: int, nxt: int) -> None:
        self.launch(slot, slot)

    def timings(self):
        return [0.0, 0.0, 0.0, 0.0]

    def launch(self, slot: int, oslot: int) -> None:
        self._arena[:] = self._in[slot]
        if self.tp_world > 1:
            self._bcast()
        self._run(self.outputs[oslot])

    def worker_loop(self) -> None:
        while True:
            self._bcast()
            kind = int(self._av["hdr"][H_KIND])
            if kind == KIND_STOP:
                return
            if kind == KIND_CAPTURE:
                self._graphs.add(int(self._av["hdr"][H_BUCKET]))
                continue
            self._run(None)

    def _run(self, out: Optional[Dict[str, np.ndarray]]) -> None:
        a = self._av
        h = a["hdr"]
        nc = int(h[H_NCOPY])
        if nc:   # prefix-cache KV block copies, ahead of the forward (runner.hip run())
            src = torch.from_numpy(a["kvcopy"][:nc, 0].astype(np.int64)).to(self.device)
            dst = torch.from_numpy(a["kvcopy"][:nc, 1].astype(np.int64)).to(self.device)
            for kc, vc in self.kv:
                kc[dst] = kc[src]
                vc[dst] = vc[src]
        T, nd, nps, ntiles, nrows = (int(h[i]) for i in (H_T, H_ND, H_NPS, H_NTILES, H_NROWS))
        ng, ndl, ntop, bucket = int(h[H_NGATHER]), int(h[H_NDELTA]), int(h[H_NTOP]), int(h[H_BUCKET])
        ids = a["ids"][:T].copy()
        if ng:
            ids[a["gdst"][:ng]] = self._tok[a["gsrc"][:ng]]
        if bucket:  # graph steps run padded to the bucket, like the captured graph
            T = nd = bucket
            ids = np.concatenate([ids, np.zeros(bucket - len(ids), np.int32)])
        dev = self.device
        tt = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
        meta = AttnMeta(positions=tt(a["pos"][:T]), slots=tt(a["slots"][:T]), num_decode=nd,
                        d_block_tables=tt(a["dbt"][:nd]) if nd else None, d_ctx_lens=tt(a["dctx"][:nd]) if nd else None,
                        nsplit=self.nsplit, blocks_per_split=self.bps, workspace=self._ws, num_prefill_tokens=T - nd,
                        p_block_tables=tt(a["pbt"][:nps]) if nps else None,
                        q_start=tt(a["q_start"][:nps]) if nps else None, q_len=tt(a["q_len"][:nps]) if nps else None,
                        ctx_len=tt(a["ctx_len"][:nps]) if nps else None,
                        tiles=tt(a["tiles"][:ntiles]) if nps else None)
        rows = None if (h[H_ROWS_ALL] or bucket) else tt(a["rows"][:nrows])
        tp = self.model.tp
        vp = tp.world > 1   # vocab-parallel sampling: no logit all-gather
        logits = self.model.forward_logits(tt(ids), meta, self.kv, rows, local=vp)
        if nrows == 0:
            return
        logits = logits[:nrows].float().clone()
        voff = self.model.vocab_start if vp else 0
        for r, t, v in a["deltas"][:ndl]:
            if 0 <= int(t) - voff < logits.shape[1]:
                logits[int(r), int(t) - voff] += float(np.array(v, np.int32).view(np.float32))
        args = (tt(a["temp"][:nrows]), tt(a["top_k"][:nrows]), tt(a["top_p"][:nrows]), tt(a["seeds"][:nrows]),
                tt(a["steps"][:nrows]))
        if vp:
            tok, lp, ti, tl = ops.sample_vocab_parallel(logits, voff, self.model.cfg.vocab_size, *args, n_top=ntop,
                                                        group=tp.group, world=tp.world)
        else:
            tok, lp, ti, tl = ops.sample(logits, *args, n_top=ntop)
        self._tok[:nrows] = tok.cpu().numpy()
        if out is not None:
            out["tok"][:nrows] = self._tok[:nrows]
            out["lp"][:nrows] = lp.cpu().numpy()
            if ntop:
                out["ti"][: nrows * ntop] = ti.cpu().numpy().reshape(-1)
                out["tl"][: nrows * ntop] = tl.cpu().numpy().reshape(-1)
