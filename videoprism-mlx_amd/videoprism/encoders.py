"""FactorizedEncoder host object backed by libvideoprism_hip.so.

Mirrors the reference module `encoders.FactorizedEncoder` (encoders.py:391-580) as used
through Flax: attributes = the CONFIGS keys, `init(rng, inputs, train=False)` returns
{'params': tree} and `apply(variables, inputs, train=False, return_intermediate=False,
frame_paddings=None)` returns `(embeddings [B, T*N, D], outputs)`.  All arithmetic runs
in the HIP kernels behind the C-ABI; this file only moves parameters and buffers.
"""

from __future__ import annotations

import ctypes
import dataclasses
from collections.abc import Collection
from typing import Any

import numpy as np

from . import _native
from . import params as params_lib


def _contains(collection, key: str) -> bool:
    """encoders.py:36-47."""
    return collection if isinstance(collection, bool) else key in collection


def _torch():
    import torch
    return torch


def _is_bf16_dtype(dt) -> bool:
    if dt is None:
        return False
    name = getattr(dt, "name", None) or getattr(dt, "__name__", None) or str(dt)
    return "bfloat16" in str(name) or "bfloat16" in str(dt)


class Engine:
    """One vp_handle (packed weights on one device) plus a reusable workspace."""

    def __init__(self, cfg: dict, flat_params: dict, device: int, bf16: bool):
        self.cfg = dict(cfg)
        self.device = device
        self.bf16 = bf16
        lib = _native.load()
        c = _native.vp_config(
            patch_size=cfg["patch_size"], pos_emb_t=cfg["pos_emb_shape"][0],
            pos_emb_h=cfg["pos_emb_shape"][1], pos_emb_w=cfg["pos_emb_shape"][2],
            model_dim=cfg["model_dim"], num_spatial_layers=cfg["num_spatial_layers"],
            num_temporal_layers=cfg["num_temporal_layers"], num_heads=cfg["num_heads"],
            mlp_dim=cfg["mlp_dim"], atten_logit_cap=float(cfg.get("atten_logit_cap", 0.0)),
            fprop_dtype=_native.VP_BF16 if bf16 else _native.VP_F32)
        h = ctypes.c_void_p()
        _native.check(lib.vp_create(ctypes.byref(c), device, ctypes.byref(h)))
        self._h = h
        try:
            for name, arr in flat_params.items():
                a = np.ascontiguousarray(arr, dtype=np.float32)
                shape = (ctypes.c_int64 * a.ndim)(*a.shape)
                _native.check(lib.vp_set_param(h, name.encode(), a.ctypes.data_as(ctypes.c_void_p),
                                               shape, a.ndim))
            _native.check(lib.vp_finalize(h))
        except Exception:
            lib.vp_destroy(h)
            self._h = None
            raise
        self._ws = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _native._lib is not None:
            _native._lib.vp_destroy(h)
            self._h = None

    # -- live per-kernel timing (HIP events on the launch stream, vp_profile_*) ---------
    def profile_enable(self, capacity: int) -> None:
        _native.call("vp_profile_enable", self._h, int(capacity))

    def profile_read(self) -> dict:
        lib = _native.load()
        n = lib.vp_profile_class_count()
        ms = (ctypes.c_double * n)()
        fl = (ctypes.c_double * n)()
        by = (ctypes.c_double * n)()
        la = (ctypes.c_int64 * n)()
        _native.call("vp_profile_read", self._h, n, ms, fl, by, la)
        out = {}
        for i in range(n):
            name = ctypes.c_char_p()
            _native.call("vp_profile_class_name", i, ctypes.byref(name))
            if la[i]:
                out[name.value.decode()] = dict(ms=ms[i], flops=fl[i], bytes=by[i], launches=la[i])
        return out

    def workspace(self, B, T, H, W):
        torch = _torch()
        n = ctypes.c_size_t()
        _native.call("vp_workspace_bytes", self._h, B, T, H, W, ctypes.byref(n))
        if self._ws is None or self._ws.numel() < n.value:
            self._ws = None
            self._ws = torch.empty(max(n.value, 256), dtype=torch.uint8,
                                   device=f"cuda:{self.device}")
        return self._ws

    def forward(self, video, frame_paddings=None, out_dtype=None, want_spatial=False,
                out=None, stream=None):
        """video: CUDA tensor [B,T,H,W,3] (fp32 or bf16) on this engine's device."""
        torch = _torch()
        if video.dim() != 5:
            raise ValueError(f"inputs must be [B, T, H, W, 3], got {tuple(video.shape)}")
        B, T, H, W, C = video.shape
        if C != 3:
            raise ValueError("inputs must have 3 channels")
        video = video.contiguous()
        in_dt = _native.VP_BF16 if video.dtype == torch.bfloat16 else _native.VP_F32
        if video.dtype not in (torch.bfloat16, torch.float32):
            video = video.float()
        out_dtype = out_dtype or (torch.bfloat16 if self.bf16 else torch.float32)
        P = self.cfg["patch_size"]
        if H % P or W % P:
            raise ValueError(f"Image height ({H}) and width ({W}) should be multiples "
                             f"of patch_size ({P}).")
        N = (H // P) * (W // P)
        D = self.cfg["model_dim"]
        if out is None:
            out = torch.empty((B, T * N, D), dtype=out_dtype, device=video.device)
        sp = torch.empty_like(out) if want_spatial else None
        fp = None
        if frame_paddings is not None:
            fp = frame_paddings.to(device=video.device, dtype=torch.float32).contiguous()
            if tuple(fp.shape) != (B, T):
                raise AssertionError(f"frame_paddings.shape == {(B, T)} failed (encoders.py:442)")
        ws = self.workspace(B, T, H, W)
        s = stream if stream is not None else torch.cuda.current_stream(video.device)
        _native.call("vp_forward", self._h, ctypes.c_void_p(video.data_ptr()), in_dt, B, T, H, W,
                     None if fp is None else ctypes.c_void_p(fp.data_ptr()),
                     ctypes.c_void_p(out.data_ptr()),
                     _native.VP_BF16 if out.dtype == torch.bfloat16 else _native.VP_F32,
                     None if sp is None else ctypes.c_void_p(sp.data_ptr()),
                     ctypes.c_void_p(ws.data_ptr()), ws.numel(), ctypes.c_void_p(s.cuda_stream))
        return out, sp


@dataclasses.dataclass
class FactorizedEncoder:
    """encoders.py:391-408 attributes; `fprop_dtype` as set by models.get_model."""

    patch_size: int = 18
    pos_emb_shape: tuple = (16, 16, 16)
    model_dim: int = 768
    num_spatial_layers: int = 12
    num_temporal_layers: int = 4
    num_heads: int = 12
    mlp_dim: int = 3072
    atten_logit_cap: float = 0.0
    norm_policy: str = "pre"
    scan: bool = False
    fprop_dtype: Any = None
    dtype: Any = None

    def __post_init__(self):
        self._engines: dict = {}

    # -- config view ---------------------------------------------------------------
    def config(self) -> dict:
        return dict(patch_size=self.patch_size, pos_emb_shape=tuple(self.pos_emb_shape),
                    model_dim=self.model_dim, num_spatial_layers=self.num_spatial_layers,
                    num_temporal_layers=self.num_temporal_layers, num_heads=self.num_heads,
                    mlp_dim=self.mlp_dim, atten_logit_cap=self.atten_logit_cap)

    def param_specs(self) -> dict:
        return params_lib.encoder_leaf_specs(self.config(), scan=True)

    @property
    def is_bf16(self) -> bool:
        return _is_bf16_dtype(self.fprop_dtype)

    # -- Flax-style API ------------------------------------------------------------
    def init(self, rng=0, inputs=None, train: bool = False, **kwargs) -> dict:
        """Returns {'params': tree} with Flax's initialiser distributions."""
        del inputs, train, kwargs
        seed = int(np.asarray(rng).ravel()[-1]) if not isinstance(rng, int) else rng
        return params_lib.flax_default_init(self.config(), seed)

    def engine(self, variables, device: int) -> Engine:
        p = variables["params"] if isinstance(variables, dict) and "params" in variables else variables
        key = (id(p), device, self.is_bf16)
        ent = self._engines.get(key)
        if ent is not None and ent[0] is p:
            return ent[1]
        if self.norm_policy != "pre":
            raise NotImplementedError("only norm_policy='pre' is implemented (all public configs)")
        flat = params_lib.canonical_params(variables)
        params_lib.validate(flat, self.param_specs())
        eng = Engine(self.config(), flat, device, self.is_bf16)
        self._engines[key] = (p, eng)
        return eng

    def apply(self, variables, inputs, train: bool = False,
              return_intermediate: bool | Collection[str] = False, frame_paddings=None,
              **kwargs):
        """encoders.py:411-456.  `train` has no effect at inference (dropouts are 0)."""
        del train
        if kwargs.get("method") not in (None,):
            raise NotImplementedError("apply(method=...) is not supported")
        torch = _torch()
        as_numpy = not isinstance(inputs, torch.Tensor)
        if as_numpy:
            x = torch.from_numpy(np.ascontiguousarray(np.asarray(inputs, dtype=np.float32)))
            device = torch.cuda.current_device()
            x = x.to(f"cuda:{device}")
        else:
            x = inputs
            if not x.is_cuda:
                x = x.to(f"cuda:{torch.cuda.current_device()}")
            device = x.device.index
        if x.dim() != 5:
            raise ValueError(f"inputs must be [B, T, H, W, 3], got {tuple(x.shape)}")
        b, t, h, w, _ = x.shape
        assert h == w  # encoders.py:435
        if self.is_bf16 and x.dtype == torch.float32:
            x = x.to(torch.bfloat16)  # colab usage: inputs cast to fprop dtype by the caller
        fp = None
        if frame_paddings is not None:
            fp = frame_paddings if isinstance(frame_paddings, torch.Tensor) else \
                torch.from_numpy(np.asarray(frame_paddings, dtype=np.float32))
        eng = self.engine(variables, device)
        want_sp = _contains(return_intermediate, "spatial_features")
        emb, sp = eng.forward(x, frame_paddings=fp, want_spatial=want_sp)
        outputs = {}
        if want_sp:
            outputs["spatial_features"] = sp
        if as_numpy:
            emb = emb.float().cpu().numpy()
            outputs = {k: v.float().cpu().numpy() for k, v in outputs.items()}
        return emb, outputs

    __call__ = apply
