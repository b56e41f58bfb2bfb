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


def _check_device(t, device: int, what: str) -> None:
    """Tensors handed to the C-ABI must live on the handle's device (raw pointers + its stream)."""
    if not t.is_cuda or t.device.index != device:
        raise ValueError(f"{what} must be on cuda:{device} (the engine's device), got {t.device}")


def _profile_enable(handle, capacity: int) -> None:
    _native.call("vp_profile_enable", handle, int(capacity))


def _profile_set_mask(handle, names=None) -> None:
    """Restrict events to the named kernel classes (None: all)."""
    mask = 0xFFFFFFFF
    if names is not None:
        lib = _native.load()
        mask = 0
        for i in range(lib.vp_profile_class_count()):
            name = ctypes.c_char_p()
            _native.call("vp_profile_class_name", i, ctypes.byref(name))
            if name.value.decode() in names:
                mask |= 1 << i
    _native.call("vp_profile_set_mask", handle, mask)


def _profile_read(handle) -> dict:
    """{kernel class: {ms, flops, bytes, launches}} since the previous read (vp_profile_read)."""
    lib = _native.load()
    n = lib.vp_profile_class_count()
    ms = (ctypes.c_double * n)()
    fl = (ctypes.c_double * n)()
    by = (ctypes.c_double * n)()
    la = (ctypes.c_int64 * n)()
    _native.call("vp_profile_read", handle, n, ms, fl, by, la)
    out = {}
    for i in range(n):
        name = ctypes.c_char_p()
        _native.call("vp_profile_class_name", i, ctypes.byref(name))
        if la[i]:
            out[name.value.decode()] = dict(ms=ms[i], flops=fl[i], bytes=by[i], launches=la[i])
    return out


def _prepare_shape(handle, seen: set, H: int, W: int, T: int) -> None:
    """First sight of a frame size / clip length: the interpolated spatial (encoders.py:497-512)
    and temporal (:543-553) positional tables, cached on the device by the library (the
    forward itself never allocates)."""
    if (H, W) not in seen:
        _native.call("vp_prepare_geometry", handle, H, W)
        seen.add((H, W))
    if T not in seen:
        _native.call("vp_prepare_frames", handle, T)
        seen.add(T)


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
        self._grids = set()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _native._lib is not None:
            _native._lib.vp_destroy(h)
            self._h = None

    # -- live per-kernel timing (HIP events on the launch stream, vp_profile_*) ---------
    def profile_enable(self, capacity: int) -> None:
        _profile_enable(self._h, capacity)

    def profile_read(self) -> dict:
        return _profile_read(self._h)

    def profile_only(self, names=None) -> None:
        _profile_set_mask(self._h, names)

    def kernel_name(self, cls_name: str) -> str:
        """Short symbol of the kernel behind profiler class `cls_name` (last launch)."""
        return _native.profile_kernel_name(self._h, cls_name)

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
        _check_device(video, self.device, "video")
        video = video.contiguous()
        if video.dtype not in (torch.bfloat16, torch.float32, torch.uint8):
            video = video.float()
        in_dt = _native._prec(video)  # uint8 frames are normalised /255 on device
        out_dtype = out_dtype or (torch.bfloat16 if self.bf16 else torch.float32)
        P = self.cfg["patch_size"]
        if H % P or W % P:
            raise ValueError(f"Image height ({H}) and width ({W}) should be multiples "
                             f"of patch_size ({P}).")
        N = (H // P) * (W // P)
        D = self.cfg["model_dim"]
        _prepare_shape(self._h, self._grids, H, W, T)
        if out is None:
            out = torch.empty((B, T * N, D), dtype=out_dtype, device=video.device)
        else:  # the kernels write B*T*N*D elements through the raw pointer
            _check_device(out, self.device, "out")
            if tuple(out.shape) != (B, T * N, D) or out.dtype not in (torch.bfloat16, torch.float32) \
                    or not out.is_contiguous():
                raise ValueError(f"out must be a contiguous bf16/fp32 tensor of shape {(B, T * N, D)}, "
                                 f"got {tuple(out.shape)} {out.dtype} contiguous={out.is_contiguous()}")
        sp = torch.empty_like(out) if want_spatial else None
        fp = None
        if frame_paddings is not None:
            fp = frame_paddings.to(device=video.device, dtype=torch.float32).contiguous()
            if tuple(fp.shape) != (B, T):
                raise AssertionError(f"frame_paddings.shape == {(B, T)} failed (encoders.py:442)")
        if B == 0:  # an empty batch: the reference's zero-size result, nothing to launch
            return out, sp
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
            arr = np.asarray(inputs)
            # uint8 frames travel as bytes (4x less H2D than fp32) and are normalised /255 on
            # device exactly as video_utils.py:94
            x = torch.from_numpy(np.ascontiguousarray(arr if arr.dtype == np.uint8 else
                                                      arr.astype(np.float32, copy=False)))
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


class ClipEngine:
    """One vp_clip handle (packed LvT weights on one device) plus reusable workspaces."""

    def __init__(self, cfg: dict, flat_params: dict, device: int, bf16: bool):
        self.cfg = dict(cfg)
        self.device = device
        self.bf16 = bf16
        lib = _native.load()
        v = _native.vp_config(
            patch_size=cfg["patch_size"], pos_emb_t=cfg["pos_emb_shape"][0],
            pos_emb_h=cfg["pos_emb_shape"][1], pos_emb_w=cfg["pos_emb_shape"][2],
            model_dim=cfg["model_dim"], num_spatial_layers=cfg["num_spatial_layers"],
            num_temporal_layers=cfg["num_temporal_layers"], num_heads=cfg["num_heads"],
            mlp_dim=cfg["mlp_dim"], atten_logit_cap=float(cfg.get("atten_logit_cap", 0.0)),
            fprop_dtype=_native.VP_BF16 if bf16 else _native.VP_F32)
        c = _native.vp_clip_config(
            video=v, num_auxiliary_layers=cfg.get("num_auxiliary_layers", 0),
            vocabulary_size=cfg["vocabulary_size"],
            num_unimodal_layers=cfg["num_unimodal_layers"],
            enable_causal_atten=1 if cfg.get("enable_causal_atten", True) else 0)
        h = ctypes.c_void_p()
        _native.check(lib.vp_clip_create(ctypes.byref(c), device, ctypes.byref(h)))
        self._h = h
        try:
            for name, arr in flat_params.items():
                a = np.ascontiguousarray(arr, dtype=np.float32)
                shape = (ctypes.c_int64 * a.ndim)(*a.shape)
                _native.check(lib.vp_clip_set_param(h, name.encode(),
                                                    a.ctypes.data_as(ctypes.c_void_p), shape, a.ndim))
            _native.check(lib.vp_clip_finalize(h))
        except Exception:
            lib.vp_clip_destroy(h)
            self._h = None
            raise
        self._ws = {}
        self._grids = set()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _native._lib is not None:
            _native._lib.vp_clip_destroy(h)
            self._h = None

    def video_handle(self):
        v = ctypes.c_void_p()
        _native.call("vp_clip_video_handle", self._h, ctypes.byref(v))
        return v

    def profile_enable(self, capacity: int) -> None:
        """HIP events around every launch of both towers (vision, auxiliary, pooler, text)."""
        _profile_enable(self.video_handle(), capacity)

    def profile_read(self) -> dict:
        return _profile_read(self.video_handle())

    def profile_only(self, names=None) -> None:
        _profile_set_mask(self.video_handle(), names)

    def kernel_name(self, cls_name: str) -> str:
        return _native.profile_kernel_name(self.video_handle(), cls_name)

    def _workspace(self, key, nbytes):
        torch = _torch()
        ws = self._ws.get(key)
        if ws is None or ws.numel() < nbytes:
            self._ws[key] = None
            ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=f"cuda:{self.device}")
            self._ws[key] = ws
        return ws

    def encode_video(self, video, frame_paddings=None, normalize=True, want_frames=False,
                     want_spatial=False, want_spatiotemporal=False, stream=None):
        torch = _torch()
        B, T, H, W, C = video.shape
        if C != 3:
            raise ValueError("inputs must have 3 channels")
        P = self.cfg["patch_size"]
        if H % P or W % P:
            raise ValueError(f"Image height ({H}) and width ({W}) should be multiples "
                             f"of patch_size ({P}).")
        _check_device(video, self.device, "video")
        video = video.contiguous()
        if video.dtype not in (torch.bfloat16, torch.float32, torch.uint8):
            video = video.float()
        in_dt = _native._prec(video)  # uint8 frames are normalised /255 on device
        D = self.cfg["model_dim"]
        N = (H // P) * (W // P)
        _prepare_shape(self.video_handle(), self._grids, H, W, T)
        fdt = torch.bfloat16 if self.bf16 else torch.float32
        dev = video.device
        vemb = torch.empty((B, D), dtype=torch.float32, device=dev)
        femb = torch.empty((B, T, D), dtype=torch.float32, device=dev) if want_frames else None
        sp = torch.empty((B, T * N, D), dtype=fdt, device=dev) if want_spatial else None
        st = torch.empty((B, T * N, D), dtype=fdt, device=dev) if want_spatiotemporal else None
        fp = None
        if frame_paddings is not None:
            fp = frame_paddings.to(device=dev, dtype=torch.float32).contiguous()
            if tuple(fp.shape) != (B, T):
                raise AssertionError(f"frame_paddings.shape == {(B, T)} failed (encoders.py:442)")
        if B == 0:  # an empty batch: zero-size embeddings, nothing to launch
            return vemb, femb, sp, st
        n = ctypes.c_size_t()
        _native.call("vp_clip_video_workspace_bytes", self._h, B, T, H, W, ctypes.byref(n))
        ws = self._workspace("video", n.value)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _native.call("vp_clip_encode_video", self._h, ptr(video), in_dt, B, T, H, W, ptr(fp),
                     1 if normalize else 0, ptr(vemb), ptr(femb), ptr(sp), ptr(st),
                     _native.VP_BF16 if self.bf16 else _native.VP_F32, ptr(ws), ws.numel(),
                     ctypes.c_void_p(s.cuda_stream))
        return vemb, femb, sp, st

    def encode_text(self, ids, paddings, normalize=True, stream=None):
        torch = _torch()
        Q, L = ids.shape
        _check_device(ids, self.device, "text_token_ids")
        ids = ids.to(dtype=torch.int32).contiguous()
        pad = paddings.to(device=ids.device, dtype=torch.float32).contiguous()
        if tuple(pad.shape) != (Q, L):
            raise ValueError(f"text_paddings must be [{Q}, {L}], got {tuple(pad.shape)}")
        D = self.cfg["model_dim"]
        out = torch.empty((Q, D), dtype=torch.float32, device=ids.device)
        if Q == 0 and L >= 1:  # no queries: a zero-size result, nothing to launch
            return out
        n = ctypes.c_size_t()
        _native.call("vp_clip_text_workspace_bytes", self._h, Q, L, ctypes.byref(n))
        ws = self._workspace("text", n.value)
        s = stream if stream is not None else torch.cuda.current_stream(ids.device)
        _native.call("vp_clip_encode_text", self._h, ctypes.c_void_p(ids.data_ptr()),
                     ctypes.c_void_p(pad.data_ptr()), Q, L, 1 if normalize else 0,
                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ws.numel(),
                     ctypes.c_void_p(s.cuda_stream))
        return out


@dataclasses.dataclass
class FactorizedVideoCLIP:
    """encoders.py:762-910 attributes (the LvT video-text model); `fprop_dtype` as set by
    models.get_model."""

    patch_size: int = 18
    pos_emb_shape: tuple = (16, 16, 16)
    num_spatial_layers: int = 12
    num_temporal_layers: int = 4
    mlp_dim: int = 3072
    num_auxiliary_layers: int = 0
    vocabulary_size: int = 128
    enable_causal_atten: bool = True
    num_unimodal_layers: int = 12
    norm_policy: str = "pre"
    model_dim: int = 768
    num_heads: int = 12
    atten_logit_cap: float = 0.0
    scan: bool = False
    fprop_dtype: Any = None
    dtype: Any = None

    def __post_init__(self):
        self._engines: dict = {}

    def config(self) -> dict:
        return dict(patch_size=self.patch_size, pos_emb_shape=tuple(self.pos_emb_shape),
                    num_spatial_layers=self.num_spatial_layers,
                    num_temporal_layers=self.num_temporal_layers, mlp_dim=self.mlp_dim,
                    num_auxiliary_layers=self.num_auxiliary_layers,
                    vocabulary_size=self.vocabulary_size,
                    enable_causal_atten=self.enable_causal_atten,
                    num_unimodal_layers=self.num_unimodal_layers, model_dim=self.model_dim,
                    num_heads=self.num_heads, atten_logit_cap=self.atten_logit_cap)

    def param_specs(self) -> dict:
        return params_lib.clip_leaf_specs(self.config(), scan=True)

    @property
    def is_bf16(self) -> bool:
        return _is_bf16_dtype(self.fprop_dtype)

    def init(self, rng=0, inputs=None, train: bool = False, **kwargs) -> dict:
        del inputs, train, kwargs
        seed = int(np.asarray(rng).ravel()[-1]) if not isinstance(rng, int) else rng
        return params_lib.synthetic_params(self.config(), seed, specs=self.param_specs())

    def engine(self, variables, device: int) -> ClipEngine:
        p = variables["params"] if isinstance(variables, dict) and "params" in variables else variables
        key = (id(p), device, self.is_bf16)
        ent = self._engines.get(key)
        if ent is not None and ent[0] is p:
            return ent[1]
        if self.norm_policy != "pre":
            raise NotImplementedError("only norm_policy='pre' is implemented (public LvT configs)")
        flat = params_lib.canonical_params(variables)
        params_lib.validate(flat, self.param_specs())
        eng = ClipEngine(self.config(), flat, device, self.is_bf16)
        self._engines[key] = (p, eng)
        return eng

    def apply(self, variables, inputs=None, text_token_ids=None, text_paddings=None,
              train: bool = False, normalize: bool = True,
              return_intermediate: bool | Collection[str] = False, frame_paddings=None, **kwargs):
        """encoders.py:788-910 -> (video_embeddings [B, D] | None, text_embeddings [B, D] | None,
        outputs).  Embeddings are returned in the fprop dtype (encoders.py:50-67 casts the
        normalised fp32 vector back)."""
        del train
        if kwargs.get("method") not in (None,):
            raise NotImplementedError("apply(method=...) is not supported")
        torch = _torch()
        as_numpy = not any(isinstance(t, torch.Tensor) for t in (inputs, text_token_ids)
                           if t is not None)
        device = torch.cuda.current_device()
        for t in (inputs, text_token_ids):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                device = t.device.index
        eng = self.engine(variables, device)
        dev = f"cuda:{device}"
        fdt = torch.bfloat16 if self.is_bf16 else torch.float32
        video_emb = text_emb = None
        outputs = {}
        if inputs is not None:
            if isinstance(inputs, torch.Tensor):
                x = inputs
            else:
                arr = np.asarray(inputs)
                x = torch.from_numpy(np.ascontiguousarray(
                    arr if arr.dtype == np.uint8 else arr.astype(np.float32, copy=False)))
            x = x.to(dev)
            if x.dim() != 5:
                raise ValueError(f"inputs must be [B, T, H, W, 3], got {tuple(x.shape)}")
            assert x.shape[2] == x.shape[3]  # encoders.py:435
            if self.is_bf16 and x.dtype == torch.float32:
                x = x.to(torch.bfloat16)
            fp = None
            if frame_paddings is not None:
                fp = frame_paddings if isinstance(frame_paddings, torch.Tensor) else \
                    torch.from_numpy(np.asarray(frame_paddings, dtype=np.float32))
            vemb, femb, sp, st = eng.encode_video(
                x, fp, normalize, want_frames=_contains(return_intermediate, "frame_embeddings"),
                want_spatial=_contains(return_intermediate, "spatial_features"),
                want_spatiotemporal=_contains(return_intermediate, "spatiotemporal_features"))
            video_emb = vemb.to(fdt)
            for k, v in (("spatial_features", sp), ("spatiotemporal_features", st),
                         ("frame_embeddings", femb)):
                if v is not None:
                    outputs[k] = v.to(fdt)
        if text_token_ids is not None:
            assert text_paddings is not None, "Text paddings are required."
            ids = text_token_ids if isinstance(text_token_ids, torch.Tensor) else \
                torch.from_numpy(np.asarray(text_token_ids, dtype=np.int32))
            pads = text_paddings if isinstance(text_paddings, torch.Tensor) else \
                torch.from_numpy(np.asarray(text_paddings, dtype=np.float32))
            text_emb = eng.encode_text(ids.to(dev), pads.to(dev), normalize).to(fdt)
        if as_numpy:
            cvt = lambda t: None if t is None else t.float().cpu().numpy()  # noqa: E731
            video_emb, text_emb = cvt(video_emb), cvt(text_emb)
            outputs = {k: cvt(v) for k, v in outputs.items()}
        return video_emb, text_emb, outputs

    __call__ = apply


class ClassifierEngine:
    """One vp_classifier handle (FactorizedVideoClassifier weights on one device)."""

    def __init__(self, cfg: dict, num_classes: int, flat_params: dict, device: int, bf16: bool):
        self.cfg = dict(cfg)
        self.num_classes = num_classes
        self.device = device
        self.bf16 = bf16
        lib = _native.load()
        v = _native.vp_config(
            patch_size=cfg["patch_size"], pos_emb_t=cfg["pos_emb_shape"][0],
            pos_emb_h=cfg["pos_emb_shape"][1], pos_emb_w=cfg["pos_emb_shape"][2],
            model_dim=cfg["model_dim"], num_spatial_layers=cfg["num_spatial_layers"],
            num_temporal_layers=cfg["num_temporal_layers"], num_heads=cfg["num_heads"],
            mlp_dim=cfg["mlp_dim"], atten_logit_cap=float(cfg.get("atten_logit_cap", 0.0)),
            fprop_dtype=_native.VP_BF16 if bf16 else _native.VP_F32)
        h = ctypes.c_void_p()
        _native.check(lib.vp_classifier_create(ctypes.byref(v), num_classes, device, ctypes.byref(h)))
        self._h = h
        try:
            for name, arr in flat_params.items():
                a = np.ascontiguousarray(arr, dtype=np.float32)
                shape = (ctypes.c_int64 * a.ndim)(*a.shape)
                _native.check(lib.vp_classifier_set_param(h, name.encode(),
                                                          a.ctypes.data_as(ctypes.c_void_p), shape,
                                                          a.ndim))
            _native.check(lib.vp_classifier_finalize(h))
        except Exception:
            lib.vp_classifier_destroy(h)
            self._h = None
            raise
        self._ws = None
        self._grids = set()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _native._lib is not None:
            _native._lib.vp_classifier_destroy(h)
            self._h = None

    def video_handle(self):
        v = ctypes.c_void_p()
        _native.call("vp_classifier_video_handle", self._h, ctypes.byref(v))
        return v

    def forward(self, video, frame_paddings=None, want_embeddings=False, want_spatial=False,
                want_spatiotemporal=False, stream=None):
        torch = _torch()
        B, T, H, W, C = video.shape
        P = self.cfg["patch_size"]
        if C != 3:
            raise ValueError("inputs must have 3 channels")
        if H % P or W % P:
            raise ValueError(f"Image height ({H}) and width ({W}) should be multiples "
                             f"of patch_size ({P}).")
        _check_device(video, self.device, "video")
        video = video.contiguous()
        if video.dtype not in (torch.bfloat16, torch.float32, torch.uint8):
            video = video.float()
        in_dt = _native._prec(video)
        _prepare_shape(self.video_handle(), self._grids, H, W, T)
        D, N = self.cfg["model_dim"], (H // P) * (W // P)
        dev = video.device
        fdt = torch.bfloat16 if self.bf16 else torch.float32
        logits = torch.empty((B, self.num_classes), dtype=torch.float32, device=dev)
        emb = torch.empty((B, D), dtype=torch.float32, device=dev) if want_embeddings else None
        sp = torch.empty((B, T * N, D), dtype=fdt, device=dev) if want_spatial else None
        st = torch.empty((B, T * N, D), dtype=fdt, device=dev) if want_spatiotemporal else None
        fp = None
        if frame_paddings is not None:
            fp = frame_paddings.to(device=dev, dtype=torch.float32).contiguous()
            if tuple(fp.shape) != (B, T):
                raise AssertionError(f"frame_paddings.shape == {(B, T)} failed (encoders.py:442)")
        if B == 0:  # an empty batch: zero-size logits, nothing to launch
            return logits, emb, sp, st
        n = ctypes.c_size_t()
        _native.call("vp_classifier_workspace_bytes", self._h, B, T, H, W, ctypes.byref(n))
        if self._ws is None or self._ws.numel() < n.value:
            self._ws = None
            self._ws = torch.empty(max(n.value, 256), dtype=torch.uint8, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _native.call("vp_classifier_forward", self._h, ptr(video), in_dt, B, T, H, W, ptr(fp),
                     ptr(logits), ptr(emb), ptr(sp), ptr(st),
                     _native.VP_BF16 if self.bf16 else _native.VP_F32, ptr(self._ws),
                     self._ws.numel(), ctypes.c_void_p(s.cuda_stream))
        return logits, emb, sp, st


@dataclasses.dataclass
class FactorizedVideoClassifier:
    """encoders.py:583-653: `encoder_params` (a FactorizedEncoder config) and `num_classes`."""

    encoder_params: dict = dataclasses.field(default_factory=dict)
    num_classes: int = 0
    fprop_dtype: Any = None
    dtype: Any = None

    def __post_init__(self):
        self._engines: dict = {}

    @property
    def is_bf16(self) -> bool:
        return _is_bf16_dtype(self.fprop_dtype)

    def config(self) -> dict:
        c = {k: v for k, v in self.encoder_params.items() if k not in ("scan", "norm_policy")}
        c["pos_emb_shape"] = tuple(c["pos_emb_shape"])
        return c

    def param_specs(self) -> dict:
        return params_lib.classifier_leaf_specs(self.config(), self.num_classes, scan=True)

    def init(self, rng=0, inputs=None, train: bool = False, **kwargs) -> dict:
        del inputs, train, kwargs
        seed = int(np.asarray(rng).ravel()[-1]) if not isinstance(rng, int) else rng
        return params_lib.synthetic_params(self.config(), seed, specs=self.param_specs())

    def engine(self, variables, device: int) -> ClassifierEngine:
        p = variables["params"] if isinstance(variables, dict) and "params" in variables else variables
        key = (id(p), device, self.is_bf16)
        ent = self._engines.get(key)
        if ent is not None and ent[0] is p:
            return ent[1]
        if self.encoder_params.get("norm_policy", "pre") != "pre":
            raise NotImplementedError("only norm_policy='pre' is implemented")
        flat = params_lib.canonical_params(variables)
        params_lib.validate(flat, self.param_specs())
        eng = ClassifierEngine(self.config(), self.num_classes, flat, device, self.is_bf16)
        self._engines[key] = (p, eng)
        return eng

    def apply(self, variables, inputs, train: bool = False,
              return_intermediate: bool | Collection[str] = False, frame_paddings=None, **kwargs):
        """encoders.py:594-653 -> (logits [B, num_classes], outputs)."""
        del train
        if kwargs.get("method") not in (None,):
            raise NotImplementedError("apply(method=...) is not supported")
        torch = _torch()
        as_numpy = not isinstance(inputs, torch.Tensor)
        if as_numpy:
            arr = np.asarray(inputs)
            x = torch.from_numpy(np.ascontiguousarray(
                arr if arr.dtype == np.uint8 else arr.astype(np.float32, copy=False)))
            device = torch.cuda.current_device()
        else:
            x = inputs
            device = x.device.index if x.is_cuda else torch.cuda.current_device()
        x = x.to(f"cuda:{device}")
        if x.dim() != 5:
            raise ValueError(f"inputs must be [B, T, H, W, 3], got {tuple(x.shape)}")
        assert x.shape[2] == x.shape[3]  # encoders.py:435
        if self.is_bf16 and x.dtype == torch.float32:
            x = x.to(torch.bfloat16)
        fp = None
        if frame_paddings is not None:
            fp = frame_paddings if isinstance(frame_paddings, torch.Tensor) else \
                torch.from_numpy(np.asarray(frame_paddings, dtype=np.float32))
        eng = self.engine(variables, device)
        logits, emb, sp, st = eng.forward(
            x, fp, want_embeddings=_contains(return_intermediate, "global_embeddings"),
            want_spatial=_contains(return_intermediate, "spatial_features"),
            want_spatiotemporal=_contains(return_intermediate, "spatiotemporal_features"))
        fdt = torch.bfloat16 if self.is_bf16 else torch.float32
        logits = logits.to(fdt)
        outputs = {}
        for k, v in (("spatial_features", sp), ("spatiotemporal_features", st),
                     ("global_embeddings", emb)):
            if v is not None:
                outputs[k] = v.to(fdt)
        if as_numpy:
            logits = logits.float().cpu().numpy()
            outputs = {k: v.float().cpu().numpy() for k, v in outputs.items()}
        return logits, outputs

    __call__ = apply
