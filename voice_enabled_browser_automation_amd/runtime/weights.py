"""Checkpoint loading: HF-layout safetensors shards, read lazily, one tensor at a
time, and TP-sharded/fused on load by the model classes.

The benchmark runs random-init weights (no network for checkpoints), but a deployment points
``VWA_LLM_WEIGHTS`` / ``VWA_ASR_WEIGHTS`` at a checkpoint directory:

* ``model.safetensors`` or ``model-0000x-of-0000y.safetensors`` + ``model.safetensors.index.json``;
* tensors are memory-mapped by ``safetensors.safe_open`` (nothing executes from the file), so a
  rank only materialises the layer it is slicing: peak host memory is one full layer, not the
  model (Llama-3-70B TP=8: ~1.7 GB instead of 140 GB per rank);
* every rank reads the same files and keeps its own shard (no weight broadcast over RCCL).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Iterator, List, Optional

import torch


class LazySafetensors:
    """Mapping name -> tensor over one or more safetensors files, loaded on access."""

    def __init__(self, path: str):
        from safetensors import safe_open

        files: List[str]
        if os.path.isdir(path):
            idx = os.path.join(path, "model.safetensors.index.json")
            if os.path.exists(idx):
                with open(idx) as fh:
                    wm = json.load(fh)["weight_map"]
                files = sorted(set(os.path.join(path, f) for f in wm.values()))
            else:
                files = sorted(os.path.join(path, f) for f in os.listdir(path) if f.endswith(".safetensors"))
        else:
            files = [path]
        if not files:
            raise FileNotFoundError(f"no .safetensors files under {path}")
        self._handles = [safe_open(f, framework="pt", device="cpu") for f in files]
        self._where: Dict[str, int] = {}
        for i, h in enumerate(self._handles):
            for k in h.keys():
                self._where[k] = i

    def __contains__(self, name: str) -> bool:
        return name in self._where

    def __getitem__(self, name: str) -> torch.Tensor:
        return self._handles[self._where[name]].get_tensor(name)

    def keys(self) -> Iterator[str]:
        return iter(self._where)

    def __len__(self) -> int:
        return len(self._where)


def load_llm(name: str, *, device, tp=None, seed: int = 0, weights_path: Optional[str] = None,
             wdtype: str = "bf16"):
    """Build the intent LLM of preset ``name`` (random init, or from ``weights_path``); ``wdtype``
    "fp8" quantises the Llama projections to OCP e4m3 on load."""
    from ..models.config import GPT2Config, get_config

    cfg = get_config(name)
    w = LazySafetensors(weights_path) if weights_path else None
    if isinstance(cfg, GPT2Config):
        from ..models.gpt2 import GPT2Model

        return GPT2Model(cfg, device=device, seed=seed, weights=w)
    from ..models.llama import LlamaModel

    return LlamaModel(cfg, device=device, tp=tp, seed=seed, weights=w, wdtype=wdtype)
