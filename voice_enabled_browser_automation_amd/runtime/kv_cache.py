"""Paged KV cache + ref-counted block manager with a hash-chained prefix cache (N3).

The brain's prompt is a ~1.0k-token static prefix (system prompt + 10 few-shot messages,
apps/brain/src/server.ts:13-82) followed by a short per-request suffix
(JSON.stringify({text, session_id, context}), :104).  Full blocks of every computed prompt are
registered under a chained hash (hash(parent_hash, block_tokens)), so the next request that
starts with the same tokens maps its first blocks onto the cached ones (ref-counted, never
written again: a sequence only appends into blocks it owns exclusively) and only prefills its
suffix.  Sized for 288 GB HBM per GPU: ``blocks_for_budget`` turns a byte budget (VWA_KV_GB)
into a block count.
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch


class PagedKVCache:
    """K/V storage: ``k[layer]`` is ``[num_blocks, n_kv_heads, block_size, head_dim]`` (contiguous)."""

    def __init__(self, n_layers: int, n_kv_heads: int, head_dim: int, block_size: int, num_blocks: int,
                 device="cpu", dtype=torch.bfloat16):
        self.n_layers, self.n_kv_heads, self.head_dim = n_layers, n_kv_heads, head_dim
        self.block_size, self.num_blocks = block_size, num_blocks
        shape = (n_layers, num_blocks, n_kv_heads, block_size, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)

    @staticmethod
    def bytes_per_block(n_layers: int, n_kv_heads: int, head_dim: int, block_size: int, elem: int = 2) -> int:
        return 2 * n_layers * n_kv_heads * block_size * head_dim * elem

    @staticmethod
    def blocks_for_budget(budget_bytes: float, n_layers: int, n_kv_heads: int, head_dim: int, block_size: int,
                          elem: int = 2) -> int:
        return max(4, int(budget_bytes // PagedKVCache.bytes_per_block(n_layers, n_kv_heads, head_dim, block_size,
                                                                        elem)))


def _block_hash(parent: bytes, tokens: Sequence[int]) -> bytes:
    h = hashlib.blake2b(parent, digest_size=16)
    h.update(bytes(str(list(tokens)), "ascii"))
    return h.digest()


class OutOfBlocks(RuntimeError):
    pass


class BlockManager:
    """Free-list allocator with reference counts and an LRU prefix cache of full blocks."""

    def __init__(self, num_blocks: int, block_size: int, reserve_block0: bool = True):
        self.block_size = block_size
        self.num_blocks = num_blocks
        # block 0 is a scratch block: padded graph rows point at it and may never own it
        start = 1 if reserve_block0 else 0
        self.free: List[int] = list(range(num_blocks - 1, start - 1, -1))
        self.ref = [0] * num_blocks
        self.cache: "OrderedDict[bytes, int]" = OrderedDict()  # hash -> block (LRU order)
        self.block_key: Dict[int, bytes] = {}
        self.hits = 0
        self.queries = 0

    # ------------------------------------------------------------------ allocation
    def n_free(self) -> int:
        return len(self.free) + sum(1 for b in self.cache.values() if self.ref[b] == 0)

    def _evict_one(self) -> None:
        for key, b in self.cache.items():
            if self.ref[b] == 0:
                del self.cache[key]
                del self.block_key[b]
                self.free.append(b)
                return
        raise OutOfBlocks("KV cache exhausted")

    def allocate(self, n: int) -> List[int]:
        out = []
        for _ in range(n):
            if not self.free:
                self._evict_one()
            b = self.free.pop()
            self.ref[b] = 1
            out.append(b)
        return out

    def release(self, blocks: Sequence[int]) -> None:
        for b in blocks:
            assert self.ref[b] > 0, f"double free of block {b}"
            self.ref[b] -= 1
            if self.ref[b] == 0 and b not in self.block_key:
                self.free.append(b)

    # ------------------------------------------------------------------ prefix cache
    def match_prefix(self, tokens: Sequence[int]) -> Tuple[List[int], int]:
        """Longest cached run of FULL blocks at the start of ``tokens`` (blocks are ref'd)."""
        bs = self.block_size
        parent = b""
        blocks: List[int] = []
        # never match the very last token: the model must run at least one row to produce logits
        n_full = (len(tokens) - 1) // bs
        for i in range(n_full):
            self.queries += 1
            key = _block_hash(parent, tokens[i * bs : (i + 1) * bs])
            b = self.cache.get(key)
            if b is None:
                break
            self.cache.move_to_end(key)
            self.ref[b] += 1
            self.hits += 1
            blocks.append(b)
            parent = key
        return blocks, len(blocks) * bs

    def register_prefix(self, tokens: Sequence[int], blocks: Sequence[int], n_computed: int) -> None:
        """Publish the full, computed blocks of a sequence to the prefix cache."""
        bs = self.block_size
        parent = b""
        for i in range(min(n_computed // bs, len(blocks))):
            key = _block_hash(parent, tokens[i * bs : (i + 1) * bs])
            b = blocks[i]
            if key not in self.cache:
                if b in self.block_key:  # block already published under another key
                    parent = key
                    continue
                self.cache[key] = b
                self.block_key[b] = key
            parent = key
