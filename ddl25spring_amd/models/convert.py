"""Tensor layout conversion between torch-style modules (NCHW / [out,in]) and the native
flat-store layout (NHWC [K,R,S,C] with 32-padded channels, im2col'd stems, HWC-flatten Linears).

A *mapping* is a list of ``(native_name, torch_name, kind, extra)``:
  kind "conv"   : torch [K,C,R,S]  <-> native [Kp,R,S,Cp]
  kind "stem"   : torch [K,C,k,k]  <-> native [Kp,1,1,Cpad] with channel (r*k+s)*C + c
  kind "linear" : torch [out,in]   <-> native [outp,1,1,inp]; extra=(C,H,W) if the input is an
                  NCHW flatten that is HWC-ordered natively
  kind "vec"    : torch [n]        <-> native [np] (bias / BN affine / running stats)
"""
from __future__ import annotations

import torch


def to_native(t: torch.Tensor, shape, kind: str, extra=None) -> torch.Tensor:
    out = torch.zeros(shape, dtype=torch.float32)
    t = t.detach().float().cpu()
    if kind == "conv":
        w = t.permute(0, 2, 3, 1)
        out[:w.shape[0], :, :, :w.shape[3]] = w
    elif kind == "stem":
        K, C, k, _ = t.shape
        w = t.permute(0, 2, 3, 1).reshape(K, k * k * C)
        out[:K, 0, 0, :k * k * C] = w
    elif kind == "linear":
        if extra is not None:
            C, H, W = extra
            t = t.reshape(t.shape[0], C, H, W).permute(0, 2, 3, 1).reshape(t.shape[0], -1)
        out.reshape(shape[0], -1)[:t.shape[0], :t.shape[1]] = t
    elif kind == "vec":
        out[:t.shape[0]] = t
    else:
        raise ValueError(kind)
    return out


def to_torch(n: torch.Tensor, tshape, kind: str, extra=None) -> torch.Tensor:
    n = n.detach().float().cpu()
    if kind == "conv":
        K, C, R, S = tshape
        return n[:K, :, :, :C].permute(0, 3, 1, 2).contiguous()
    if kind == "stem":
        K, C, k, _ = tshape
        return n[:K, 0, 0, :k * k * C].reshape(K, k, k, C).permute(0, 3, 1, 2).contiguous()
    if kind == "linear":
        out_f, in_f = tshape
        w = n.reshape(n.shape[0], -1)[:out_f, :in_f]
        if extra is not None:
            C, H, W = extra
            w = w.reshape(out_f, H, W, C).permute(0, 3, 1, 2).reshape(out_f, -1)
        return w.contiguous()
    if kind == "vec":
        return n[:tshape[0]].clone()
    raise ValueError(kind)


def import_torch(net, module: torch.nn.Module, mapping) -> None:
    """Copy a torch module's parameters/buffers into every client slot of ``net``."""
    tsd = dict(module.state_dict())
    st = net.store
    with torch.no_grad():
        for nname, tname, kind, extra in mapping:
            spec = st.specs[nname]
            val = to_native(tsd[tname], spec.shape, kind, extra).reshape(-1).to(st.device)
            dst = st.buffers if spec.buffer else st.data
            dst[:, spec.offset:spec.offset + spec.numel] = val
    st.sync_shadow()


def export_torch(net, module: torch.nn.Module, mapping, group: int = 0, grads: bool = False):
    """Native -> torch state dict (or grads, if ``grads``) for one client slot."""
    tsd = dict(module.state_dict())
    st = net.store
    out = {}
    for nname, tname, kind, extra in mapping:
        spec = st.specs[nname]
        if grads:
            if spec.buffer:
                continue
            src = st.grad
        else:
            src = st.buffers if spec.buffer else st.data
        n = src[group, spec.offset:spec.offset + spec.numel].reshape(spec.shape)
        out[tname] = to_torch(n, tuple(tsd[tname].shape), kind, extra)
    return out


def resnet_mapping(net) -> list:
    m = []
    for name in net.store.specs:
        parts = name.split(".")
        if name.startswith("conv1."):  # stem
            if name == "conv1.weight":
                m.append((name, "conv1.weight", "stem", None))
            else:  # conv1.bn.X
                m.append((name, "bn1." + parts[-1], "vec", None))
        elif name.startswith("fc."):
            m.append((name, name, "linear" if name.endswith("weight") else "vec", None))
        else:
            # layerL.B.{conv1,conv2,conv3,downsample}[.bn].X
            stage, blk, unit = parts[0], parts[1], parts[2]
            if unit == "downsample":
                tname = f"{stage}.{blk}.downsample." + ("0.weight" if parts[3] == "weight" else f"1.{parts[-1]}")
                kind = "conv" if parts[3] == "weight" else "vec"
            else:
                idx = unit[-1]
                if parts[3] == "weight":
                    tname, kind = f"{stage}.{blk}.{unit}.weight", "conv"
                else:
                    tname, kind = f"{stage}.{blk}.bn{idx}.{parts[-1]}", "vec"
            m.append((name, tname, kind, None))
    return m
