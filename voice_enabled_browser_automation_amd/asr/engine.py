"""ASR engine: on-node Whisper transcription (replaces the Deepgram live socket,
apps/voice/src/deepgram.ts:21-67).

`WhisperRunner` owns static decoder buffers for up to ``max_sessions`` concurrent utterances
(one row per session per step -> continuous batching across voice sessions, the DP unit of a
GPU) and captures one hipGraph per row bucket.  `AsrEngine.transcribe` runs
PCM16 -> f32 (HIP) -> log-mel (HIP) -> encoder -> cross K/V -> greedy constrained decode.
"""
from __future__ import annotations

import time
from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..models.whisper import WhisperModel

BUCKETS = (1, 2, 4, 8, 16, 32, 64)



class RunnerBuffers(SimpleNamespace):
    """The decoder step's fixed-address buffers.  Hashable by identity and weak-referenceable:
    the model's chained-launch descriptors (raw pointers into these buffers) are cached per
    buffers object in a WeakKeyDictionary (models/whisper.py _chain_descs)."""

    __hash__ = object.__hash__

    def __eq__(self, other):
        return self is other

class WhisperRunner:
    def __init__(self, model: WhisperModel, *, max_sessions: int = 4, block_size: int = 16,
                 use_graphs: Optional[bool] = None):
        cfg = model.cfg
        self.model = model
        dev = model.device
        self.device = dev
        self.max_sessions = max_sessions
        self.bs = block_size
        self.bps = (cfg.n_text_ctx + block_size - 1) // block_size  # blocks per session
        n_blocks = max_sessions * self.bps + 1
        H, hd, d = model.H, model.hd, cfg.d_model
        R = max(BUCKETS)
        i32 = dict(dtype=torch.int32, device=dev)
        b = RunnerBuffers()
        # one device block for a step's inputs (tokens | positions | seq_ids | ctx_lens | slots as
        # int64) and its pinned mirror: ONE host->device copy per step (five separate copies were
        # 7 % of the 32-session batched decode's GPU time, profiles/r4_asr_tiny_batch32_kernel_stats.md)
        b.step_in = torch.zeros(6 * R, **i32)
        b.tokens, b.positions, b.seq_ids, b.ctx_lens = (b.step_in[i * R : (i + 1) * R] for i in range(4))
        b.slots = b.step_in[4 * R :].view(torch.int64)
        b.ctx_lens.fill_(1)
        b.slots.fill_(-1)
        b.block_table = torch.zeros(max_sessions, self.bps, **i32)
        for s in range(max_sessions):
            b.block_table[s] = torch.arange(1 + s * self.bps, 1 + (s + 1) * self.bps, dtype=torch.int32)
        L = cfg.n_dec_layers
        b.k_cache = torch.zeros(L, n_blocks, H, block_size, hd, dtype=model.dtype, device=dev)
        b.v_cache = torch.zeros_like(b.k_cache)
        b.max_ctx = self.bps * block_size
        b.hidden = torch.zeros(R, d, dtype=model.dtype, device=dev)
        b.h = torch.zeros_like(b.hidden)
        b.q = torch.zeros(R, d, dtype=model.dtype, device=dev)
        b.att = torch.zeros_like(b.q)
        b.f = torch.zeros(R, cfg.ffn, dtype=model.dtype, device=dev)
        b.logits = torch.zeros(R, model.vocab_padded, dtype=torch.float32, device=dev)
        ns = max(ops.decode_n_splits(b.max_ctx), ops.decode_n_splits(cfg.n_audio_ctx))
        b.part_o = torch.zeros(R * ns * H * hd, dtype=torch.float32, device=dev)
        b.part_ml = torch.zeros(R * ns * H * 2, dtype=torch.float32, device=dev)
        b.attn_cnt = torch.zeros(R * H, dtype=torch.int32, device=dev)
        b.cross = [(torch.zeros(max_sessions, cfg.n_audio_ctx, H, hd, dtype=model.dtype, device=dev),
                    torch.zeros(max_sessions, cfg.n_audio_ctx, H, hd, dtype=model.dtype, device=dev)) for _ in range(L)]
        b.cross_table = torch.arange(max_sessions, dtype=torch.int32, device=dev)[:, None].contiguous()
        b.cross_lens = torch.full((R,), cfg.n_audio_ctx, dtype=torch.int32, device=dev)
        self.b = b
        pin = dev.type == "cuda"
        self.h_in = torch.zeros(6 * R, dtype=torch.int32, pin_memory=pin)
        self.h_i32 = self.h_in[: 4 * R].view(4, R)
        self.h_slots = self.h_in[4 * R :].view(torch.int64)
        self.h_i32[3].fill_(1)
        self.h_slots.fill_(-1)
        if use_graphs is None:
            use_graphs = ops.env_flag("VWA_HIPGRAPH")
        self.use_graphs = bool(use_graphs) and dev.type == "cuda"
        self.graphs: Dict[int, Tuple[torch.cuda.CUDAGraph, torch.Tensor]] = {}
        self.pool = None
        self._copy_done: Optional["torch.cuda.Event"] = None  # the last step's staging copy (step())

    def set_cross(self, slot: int, enc_states: torch.Tensor) -> None:
        """Compute this session's cross-attention K/V from encoder states [1, T, d]."""
        kvs = self.model.cross_kv(enc_states)
        for li, (k, v) in enumerate(kvs):
            self.b.cross[li][0][slot].copy_(k[0])
            self.b.cross[li][1][slot].copy_(v[0])

    def _fwd(self, M: int) -> torch.Tensor:
        return self.model.decode_step(self.b, M)

    def _capture(self, M: int):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fwd(M)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(g, pool=self.pool):
            out = self._fwd(M)
        self.graphs[M] = (g, out)
        return self.graphs[M]

    def step(self, rows: Sequence[Tuple[int, int, int]]) -> torch.Tensor:
        """rows: (session slot, token, position). Returns f32 logits [len(rows), vocab_padded]."""
        n = len(rows)
        M = next(bk for bk in BUCKETS if bk >= n)
        if self._copy_done is not None:
            # the previous step's pinned -> device copy may still be queued behind its forward:
            # rewriting the pinned rows before it ran would feed that step the NEXT step's tokens /
            # positions / slots (back-to-back step() calls with no host sync in between; the
            # one-launch decoder leaves the host far ahead of the GPU)
            self._copy_done.synchronize()
        hi = self.h_i32
        for i, (slot, tok, pos) in enumerate(rows):
            hi[0, i], hi[1, i], hi[2, i], hi[3, i] = tok, pos, slot, pos + 1
            blk = 1 + slot * self.bps + pos // self.bs
            self.h_slots[i] = blk * self.bs + pos % self.bs
        for i in range(n, M):
            hi[0, i], hi[1, i], hi[2, i], hi[3, i] = 0, 0, 0, 1
            self.h_slots[i] = -1
        b = self.b
        b.step_in.copy_(self.h_in, non_blocking=True)
        if self.device.type == "cuda":
            if self._copy_done is None:
                self._copy_done = torch.cuda.Event()
            self._copy_done.record()
        if self.use_graphs:
            g, out = self.graphs.get(M) or self._capture(M)
            g.replay()
        else:
            out = self._fwd(M)
        return out[:n]


class AsrEngine:
    """Whisper transcription with fixed-work decoding options for benchmarking."""

    def __init__(self, model: WhisperModel, tokenizer, *, max_sessions: int = 4, use_graphs: Optional[bool] = None):
        self.model = model
        self.tok = tokenizer
        cfg = model.cfg
        self.runner = WhisperRunner(model, max_sessions=max_sessions, use_graphs=use_graphs)
        dev = model.device
        W = (model.vocab_padded + 31) // 32
        text_ids = np.arange(model.vocab_padded) < cfg.eot
        self.mask_text = torch.from_numpy(self._pack(text_ids)).to(dev)[None]
        with_eot = text_ids.copy()
        with_eot[cfg.eot] = True
        self.mask_text_eot = torch.from_numpy(self._pack(with_eot)).to(dev)[None]
        self.d_seed = torch.zeros(1, dtype=torch.int64, device=dev)
        self.d_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.d_tok = torch.zeros(1, dtype=torch.int32, device=dev)
        self.part_val = torch.zeros(64, dtype=torch.float32, device=dev)
        self.part_idx = torch.zeros(64, dtype=torch.int32, device=dev)
        self.prompt = [cfg.sot, cfg.lang_en, cfg.transcribe, cfg.no_timestamps]
        # device-resident single-session decode loop (graphs keyed by (slot, eot allowed))
        self.loop_out = torch.zeros(max(448, cfg.n_text_ctx), dtype=torch.int32, device=dev)
        self.loop_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.loop_graphs: Dict[Tuple[int, bool, int], torch.cuda.CUDAGraph] = {}
        self.device_loop = self.runner.use_graphs and ops.env_flag("VWA_ASR_DEVICE_LOOP")
        self.last_stats: Dict[str, float] = {}
        self.free_slots = list(range(max_sessions - 1, -1, -1))

    @staticmethod
    def _pack(bits: np.ndarray) -> np.ndarray:
        n = (len(bits) + 31) // 32 * 32
        b = np.zeros(n, dtype=np.uint8)
        b[: len(bits)] = bits
        return np.packbits(b, bitorder="little").view(np.uint32).view(np.int32).copy()

    def pcm_to_audio(self, pcm: np.ndarray, rate: int = 16000) -> torch.Tensor:
        t = torch.from_numpy(np.ascontiguousarray(pcm, dtype=np.int16)).to(self.model.device, non_blocking=True)
        return ops.pcm16_to_f32(t, in_rate=rate)

    def _sample(self, logits, allow_eot: bool) -> int:
        ops.sample(logits, mask=self.mask_text_eot if allow_eot else self.mask_text, temperature=None,
                   seed=self.d_seed, step=self.d_step, out_tokens=self.d_tok, part_val=self.part_val,
                   part_idx=self.part_idx)
        return int(self.d_tok[0].item())

    # ---- device-resident greedy decode (one session): step graph = forward -> masked argmax ->
    # decode_advance (sampled token becomes the next input, position / context / KV slot move on),
    # replayed back to back; the host reads the tokens once per chunk instead of once per token
    # (measured per token before: 5 metadata copies + a host round trip, ~80 us of GPU idle)
    def _loop_step(self, slot: int, allow_eot: bool) -> None:
        r = self.runner
        b = r.b
        # whisper-large persistent decoder: embedding, layers, LM head, argmax and advance are ONE
        # launch (models/whisper.py wdec_loop_step)
        if self.model.wdec_loop_step(
                b, self.mask_text_eot if allow_eot else self.mask_text, self.d_tok, self.d_step, self.loop_out,
                self.loop_cnt, 1 + slot * r.bps):
            return
        logits = r._fwd(1)
        self._advance(logits, slot, allow_eot)

    def _advance(self, logits: torch.Tensor, slot: int, allow_eot: bool) -> None:
        b = self.runner.b
        ops.sample(logits[:1], mask=self.mask_text_eot if allow_eot else self.mask_text, temperature=None,
                   seed=self.d_seed, step=self.d_step, out_tokens=self.d_tok, part_val=self.part_val,
                   part_idx=self.part_idx)
        ops.ext().decode_advance(b.tokens, b.positions, b.ctx_lens, b.slots, self.d_tok, self.loop_out,
                                 self.loop_cnt, 1 + slot * self.runner.bps, self.runner.bs)

    LOOP_STEPS = 4  # decode steps per replayed loop graph (graph-to-graph launch gap ~10 us per replay)

    def _loop_graph(self, slot: int, allow_eot: bool, steps: int = 1) -> "torch.cuda.CUDAGraph":
        key = (slot, allow_eot, steps)
        g = self.loop_graphs.get(key)
        if g is None:
            r = self.runner
            b = r.b
            # one warm-up step with no KV write (slot -1): the session's cache holds the prompt
            b.seq_ids[:1].fill_(slot)
            b.positions[:1].fill_(0)
            b.ctx_lens[:1].fill_(1)
            b.slots[:1].fill_(-1)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._loop_step(slot, allow_eot)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            if r.pool is None:
                r.pool = torch.cuda.graph_pool_handle()
            with torch.cuda.graph(g, pool=r.pool):
                for _ in range(steps):  # identical steps: each reads what the previous advanced
                    self._loop_step(slot, allow_eot)
            self.loop_graphs[key] = g
        return g

    def _decode_device(self, slot: int, first_logits: torch.Tensor, n_max: int, exact: bool,
                       P: Optional[int] = None) -> List[int]:
        """P: the session's prompt length (SOT sequence + any forced prefix) -- the first sampled
        token sits at position P."""
        cfg = self.model.cfg
        r = self.runner
        b = r.b
        P = len(self.prompt) if P is None else P
        n_max = min(n_max, self.loop_out.numel(), r.bps * r.bs - P)
        if n_max <= 0:
            return []
        g = self._loop_graph(slot, not exact)
        K = self.LOOP_STEPS
        gk = self._loop_graph(slot, not exact, K) if K > 1 else None
        # row 0 = this session at the last prompt position; the first advance moves it to P
        b.seq_ids[:1].fill_(slot)
        b.positions[:1].fill_(P - 1)
        self.loop_cnt.zero_()
        self._advance(first_logits, slot, not exact)
        out: List[int] = []
        done = 1
        chunk = n_max if exact else 8
        while True:
            todo = min(chunk, n_max - done)
            while gk is not None and todo >= K:  # K steps per replay (never past n_max)
                gk.replay()
                done += K
                todo -= K
            for _ in range(todo):
                g.replay()
                done += 1
            toks = self.loop_out[:done].tolist()
            if not exact and cfg.eot in toks:
                return toks[: toks.index(cfg.eot)]
            if done >= n_max:
                return toks[:n_max]

    def set_cross_batch(self, slots: List[int], enc_states: torch.Tensor) -> None:
        cross = self.runner.b.cross
        s0 = slots[0]
        if list(slots) == list(range(s0, s0 + len(slots))):  # a run of slots: projected in place
            self.model.cross_kv(enc_states, out=[(k[s0 : s0 + len(slots)], v[s0 : s0 + len(slots)]) for k, v in cross])
            return
        kvs = self.model.cross_kv(enc_states)
        for li, (k, v) in enumerate(kvs):
            for i, slot in enumerate(slots):
                self.runner.b.cross[li][0][slot].copy_(k[i])
                self.runner.b.cross[li][1][slot].copy_(v[i])

    def transcribe(self, audio: torch.Tensor, *, max_tokens: int = 96, min_tokens: int = 0,
                   exact_tokens: Optional[int] = None) -> str:
        """audio: f32 16 kHz on the model device (<= 30 s).

        exact_tokens: decode exactly this many text tokens (EOT suppressed) -- fixed-work mode
        used by the benchmark so random-init weights do the same work as a real transcript.
        """
        return self.transcribe_many([audio], max_tokens=max_tokens, min_tokens=min_tokens,
                                    exact_tokens=exact_tokens)[0]

    def transcribe_many(self, audios: List[torch.Tensor], *, max_tokens: int = 96, min_tokens: int = 0,
                        exact_tokens: Optional[int] = None) -> List[str]:
        """Batch of utterances (concurrent voice sessions on this GPU): one batched encoder pass
        ([B, 3000, mels] through conv/flash-attention/GEMMs), then every decode step is one
        ragged row-per-session graph replay with one masked-argmax launch for all sessions."""
        toks = self.decode_many(audios, max_tokens=max_tokens, min_tokens=min_tokens, exact_tokens=exact_tokens)
        return [self.tok.decode(o) for o in toks]

    def max_prefix(self) -> int:
        """Longest forced text prefix decode_many keeps (the decoder's position cap minus the SOT
        prompt and one decoded token); longer prefixes are cut to this length."""
        r = self.runner
        return max(0, r.bps * r.bs - len(self.prompt) - 1)

    def decode_many(self, audios: List[torch.Tensor], prefixes: Optional[Sequence[Sequence[int]]] = None, *,
                    max_tokens: int = 96, min_tokens: int = 0, exact_tokens: Optional[int] = None) -> List[List[int]]:
        """Token ids decoded for each utterance.  ``prefixes[i]``: text tokens forced after the
        SOT sequence (a streaming session's committed transcript -- asr/streaming.py local
        agreement): they are prefilled in the same ragged prompt step as the SOT tokens and only
        the continuation is decoded; the result EXCLUDES the prefix.  A prefix longer than
        ``max_prefix()`` is cut to that length (callers build hypotheses from the cut prefix)."""
        t0 = time.perf_counter()
        m = self.model
        B = len(audios)
        if B > len(self.free_slots):
            raise RuntimeError(f"{B} utterances exceed the {len(self.free_slots)} free ASR session slots")
        prefixes = [list(p) for p in prefixes] if prefixes is not None else [[] for _ in range(B)]
        assert len(prefixes) == B
        r = self.runner
        cap = r.bps * r.bs  # decoder positions per session
        prompts = [self.prompt + p[: max(0, cap - len(self.prompt) - 1)] for p in prefixes]
        slots = [self.free_slots.pop() for _ in range(B)]
        retry = False
        try:
            mel = m.mel_batch(audios)
            enc = m.encode(mel)
            self.set_cross_batch(slots, enc)
            t_enc = time.perf_counter()
            # GPU-side decode time (prompt step + token loop): the host stamps above are taken when
            # the encoder and the cross K/V projections are LAUNCHED, so decode_ms also holds
            # whatever of them was still running; events bracket the decoder's own stream time
            ev = None
            if m.device.type == "cuda":
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            logits = self._prompt_logits(slots, prompts)
            outs: List[List[int]] = [[] for _ in range(B)]
            live = list(range(B))
            n_max = exact_tokens if exact_tokens is not None else max_tokens
            pos = [len(p) for p in prompts]  # next position per session
            limit = [min(n_max, cap - len(p)) for p in prompts]
            if B == 1 and self.device_loop and (exact_tokens is not None or min_tokens == 0) and n_max > 0:
                outs[0] = self._decode_device(slots[0], logits, limit[0], exact_tokens is not None, P=pos[0])
                live = []
            for i in range(n_max if live else 0):
                allow_eot = exact_tokens is None and i >= min_tokens
                toks = self._sample_rows(logits, allow_eot)
                nxt = []
                for j, tok in zip(live, toks):
                    if tok == m.cfg.eot or tok < 0:
                        continue
                    outs[j].append(tok)
                    if len(outs[j]) < limit[j]:
                        nxt.append(j)
                live = nxt
                if not live or i + 1 >= n_max:
                    break
                logits = self.runner.step([(slots[j], outs[j][-1], pos[j] + len(outs[j]) - 1) for j in live])
            if self._chain_failed():  # results of a timed-out chained launch are invalid: redo
                retry = True
            t_end = time.perf_counter()
            dec_gpu = None
            if ev is not None:
                ev[1].record()
                ev[1].synchronize()  # (the tokens were read back: the stream is already there)
                dec_gpu = ev[0].elapsed_time(ev[1])
            self.last_stats = dict(encode_ms=(t_enc - t0) * 1e3, decode_ms=(t_end - t_enc) * 1e3,
                                   decode_gpu_ms=dec_gpu, total_ms=(t_end - t0) * 1e3,
                                   tokens=sum(len(o) for o in outs), batch=B,
                                   prefix_tokens=sum(len(p) - len(self.prompt) for p in prompts))
            if not retry:
                return outs
        finally:
            self.free_slots.extend(slots)
        return self.decode_many(audios, prefixes, max_tokens=max_tokens, min_tokens=min_tokens,
                                exact_tokens=exact_tokens)

    def _prompt_logits(self, slots: List[int], prompts: List[List[int]]) -> torch.Tensor:
        """Prefill every session's prompt (ragged rows, <= 64 per step; a session's rows stay in
        order) and return the logits of each session's LAST prompt row, in session order."""
        R = max(BUCKETS)
        rows: List[Tuple[int, int, int]] = []
        want: List[int] = []   # row index (within the pending step) of a session's last prompt token
        got: List[torch.Tensor] = []

        def run():
            nonlocal rows, want
            if rows:
                out = self.runner.step(rows)
                if want:
                    # (clone: the logits live in the replayed graph's static output buffer)
                    got.append(out[torch.tensor(want, device=out.device)].clone())
            rows, want = [], []

        for slot, prompt in zip(slots, prompts):
            if len(rows) + len(prompt) > R and len(prompt) <= R:
                run()
            for p, t in enumerate(prompt):
                if len(rows) == R:
                    run()
                rows.append((slot, t, p))
            want.append(len(rows) - 1)
        run()
        return torch.cat(got)

    def _chain_failed(self) -> bool:
        """Health check of the chained decoder launches (models/whisper.py): a grid barrier that
        timed out (workgroups not co-resident) leaves an error word; the model then falls back to
        per-kernel launches and every captured graph is dropped."""
        m = self.model
        if getattr(m, "chain_error", None) is None or getattr(m, "_chain_disabled", False) or not m.chain_error():
            return False
        import warnings

        warnings.warn("chained Whisper decode launch timed out at a grid barrier; using per-kernel launches")
        m.disable_chain()
        self.runner.graphs.clear()
        self.loop_graphs.clear()
        return True

    def _sample_rows(self, logits: torch.Tensor, allow_eot: bool) -> List[int]:
        n = logits.shape[0]
        if n == 1:
            return [self._sample(logits, allow_eot)]
        logits = logits.contiguous()
        mask = (self.mask_text_eot if allow_eot else self.mask_text).expand(n, -1).contiguous()
        if self.d_tok.numel() < n:
            self.d_tok = torch.zeros(n, dtype=torch.int32, device=self.d_tok.device)
        part_val = torch.empty(n * 64, dtype=torch.float32, device=logits.device)
        part_idx = torch.empty(n * 64, dtype=torch.int32, device=logits.device)
        ops.sample(logits, mask=mask, temperature=None, seed=self.d_seed, step=self.d_step, out_tokens=self.d_tok,
                   part_val=part_val, part_idx=part_idx)
        return self.d_tok[:n].tolist()
