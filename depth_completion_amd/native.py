"""ctypes view of the native session (include/dcamd.h "native session", csrc/session.cpp).

The session is the sampler for hosts that are not Python (a C / C++ / Go / Rust caller links libdcamd.so
and calls dc_create / dc_load_weights / dc_complete directly; INTEGRATION.md shows the C form).  This wrapper
exists so that the tests can drive the same entry points from Python and compare them with the Python
pipeline bitwise; it moves no data itself beyond what the caller passes (device tensors).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch

from . import _lib


class SampleParams(C.Structure):
    """Mirror of ``dc_sample_params``."""

    _fields_ = [("max_depth", C.c_float), ("min_depth", C.c_float), ("norm", C.c_int), ("projection", C.c_int),
                ("inv", C.c_int), ("interp", C.c_int), ("steps", C.c_int), ("resolution", C.c_int),
                ("opt", C.c_int), ("lr_latent", C.c_double), ("lr_scaling", C.c_double), ("beta", C.c_float),
                ("use_graph", C.c_int)]

    @classmethod
    def make(cls, max_depth=120.0, min_depth=0.0, norm="const", projection="linear", inv=False,
             interp_mode="bilinear", steps=50, resolution=768, opt="adam", lr=None, beta=0.9, use_graph=True):
        p = cls()
        _lib.load().dc_sample_params_default(C.addressof(p))
        lr_latent, lr_scaling = (0.05, 0.005) if lr is None else lr
        p.max_depth, p.min_depth = float(max_depth), float(min_depth)
        p.norm = {"const": 0, "minmax": 1}[norm]
        p.projection = {"linear": 0, "log": 1, "log10": 2}[projection]
        p.inv, p.interp = int(inv), {"bilinear": 0, "nearest": 1}[interp_mode]
        p.steps, p.resolution = int(steps), int(resolution)
        p.opt = {"adam": 0, "sgd": 1, "adagrad": 2}[opt]
        p.lr_latent, p.lr_scaling, p.beta, p.use_graph = float(lr_latent), float(lr_scaling), float(beta), int(use_graph)
        return p


class NativeSession:
    """dc_create + dc_load_weights(dir, tuned table) on ``device``; calls run on the current torch stream."""

    def __init__(self, weights_dir, device="cuda:0", tuned_table: str | None = None):
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.h = C.c_void_p()
        st = self.lib.dc_create(C.addressof(self.h), self.device.index or 0)
        if st != 0:
            raise _lib.DCError(f"dc_create failed: {_lib.STATUS.get(st, st)}")
        if tuned_table is None:
            tuned_table = os.environ.get("DC_TUNED") or str(Path(__file__).resolve().parent / "tuned_gfx950.json")
        self._check(self.lib.dc_load_weights(self.h, str(weights_dir).encode(), tuned_table.encode()),
                    "dc_load_weights")

    def _check(self, status, name):
        if status != 0:
            msg = self.lib.dc_session_error(self.h)
            msg = msg.decode() if msg else ""
            if status == 1:
                raise ValueError(f"{name}: {msg}")
            raise _lib.DCError(f"{name} failed ({_lib.STATUS.get(status, status)}): {msg}")

    def close(self):
        if self.h:
            self.lib.dc_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def latent_hw(self, H, W, resolution=768):
        h, w = C.c_int(), C.c_int()
        self._check(self.lib.dc_latent_hw(H, W, resolution, C.addressof(h), C.addressof(w)), "dc_latent_hw")
        return h.value, w.value

    def encode(self, imgs, resolution=768):
        n, _, H, W = imgs.shape
        h, w = self.latent_hw(H, W, resolution)
        lat = torch.empty(n, 4, h, w, dtype=torch.bfloat16, device=self.device)
        imgs = imgs.to(self.device, torch.uint8).contiguous()
        self._check(self.lib.dc_encode(self.h, imgs.data_ptr(), n, H, W, resolution, lat.data_ptr(), self.stream),
                    "dc_encode")
        return lat

    def guided_sample(self, img_latents, sparses, noise, params: SampleParams, prev=None):
        n, _, H, W = sparses.shape
        lat = torch.empty_like(img_latents)
        aff = torch.empty(n, 2, dtype=torch.float32, device=self.device)
        sp = sparses.to(self.device, torch.float32).contiguous()
        nz = noise.to(self.device, torch.bfloat16).contiguous()
        pv = prev.to(self.device, torch.bfloat16).contiguous() if prev is not None else None
        self._check(self.lib.dc_guided_sample(self.h, img_latents.contiguous().data_ptr(), nz.data_ptr(), nz.shape[0],
                                              pv.data_ptr() if pv is not None else None, sp.data_ptr(), n, H, W,
                                              C.addressof(params), lat.data_ptr(), aff.data_ptr(), self.stream),
                    "dc_guided_sample")
        return lat, aff

    def decode_dense(self, latents, affine, sparses, params: SampleParams):
        n, _, H, W = sparses.shape
        dense = torch.empty(n, 1, H, W, dtype=torch.float32, device=self.device)
        sp = sparses.to(self.device, torch.float32).contiguous()
        self._check(self.lib.dc_decode_dense(self.h, latents.contiguous().data_ptr(), affine.contiguous().data_ptr(),
                                             sp.data_ptr(), n, H, W, C.addressof(params), dense.data_ptr(), self.stream),
                    "dc_decode_dense")
        return dense

    def complete(self, imgs, sparses, noise, params: SampleParams, prev=None):
        n, _, H, W = imgs.shape
        h, w = self.latent_hw(H, W, params.resolution)
        dense = torch.empty(n, 1, H, W, dtype=torch.float32, device=self.device)
        lat = torch.empty(n, 4, h, w, dtype=torch.bfloat16, device=self.device)
        im = imgs.to(self.device, torch.uint8).contiguous()
        sp = sparses.to(self.device, torch.float32).contiguous()
        nz = noise.to(self.device, torch.bfloat16).contiguous()
        pv = prev.to(self.device, torch.bfloat16).contiguous() if prev is not None else None
        self._check(self.lib.dc_complete(self.h, im.data_ptr(), sp.data_ptr(), n, H, W, nz.data_ptr(), nz.shape[0],
                                         pv.data_ptr() if pv is not None else None, C.addressof(params),
                                         dense.data_ptr(), lat.data_ptr(), self.stream), "dc_complete")
        return dense, lat
