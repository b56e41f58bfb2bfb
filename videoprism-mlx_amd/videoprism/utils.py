"""Checkpoint IO, mirroring videoprism/utils.py:84-169 (local files only).

`load_checkpoint` returns the nested tree that `FactorizedEncoder.apply` consumes.
Remote paths (gs://, http(s)://, s3://) are rejected: this deployment has no network
and the reference's fetch path (utils.py:122-142) needs fsspec + egress.
"""

from __future__ import annotations

import os

import numpy as np


def recover_tree(keys, values):
    """utils.py:84-105 -- nested dict from '/'-separated flat names (the reference's public
    helper; the tree itself is built by params.unflatten, the package's one implementation)."""
    from .params import unflatten
    return unflatten(dict(zip(keys, values)))


def npload(fname):
    """utils.py:145-154 — np.load without pickles; .safetensors also accepted."""
    if fname.startswith(("gs://", "http://", "https://", "s3://")):
        raise ValueError(f"remote checkpoint paths are not supported offline: {fname}")
    if fname.endswith(".safetensors"):
        from safetensors.numpy import load_file
        return dict(load_file(fname))
    loaded = np.load(fname, allow_pickle=False)
    if isinstance(loaded, np.ndarray):
        return loaded
    return dict(loaded)


def load_checkpoint(npz):
    """utils.py:157-169."""
    if isinstance(npz, (str, os.PathLike)):
        npz = npload(os.fspath(npz))
    keys, values = zip(*list(npz.items()))
    return recover_tree(keys, values)


def save_checkpoint(path, variables) -> None:
    """Writes {'params': tree} as a Flax-style '/'-keyed npz (inverse of load_checkpoint)."""
    from .params import flatten
    flat = flatten(variables)
    np.savez(path, **{k: np.asarray(v, dtype=np.float32) for k, v in flat.items()})
