"""Probe: the fp8 MFMA's product of every pair of e4m3 codes.  A 1x1 conv
with C = 64 where pixel p holds code v_p in every channel and output channel
o has code u_o in every weight: acc[o][p] = 64 * val(u_o) * val(v_p), exact
in fp32.  Any deviation shows how v_mfma_f32_32x32x64_f8f6f4 interprets the
operands.  Writes gpurun_out/f8_pair_probe.npz.  Test infrastructure only."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O  # noqa: E402
from dlq_amd import ops  # noqa: E402


def main():
    codes = np.arange(256, dtype=np.uint8)
    codes[(codes & 0x7F) == 0x7F] = 0  # no NaN operands
    C = 64
    x = np.repeat(codes[:, None], C, axis=1).reshape(1, 16, 16, C)  # NHWC, pixel p = code p
    w = np.repeat(codes[:, None], C, axis=1).reshape(256, C, 1, 1)
    packed = ops.pack_conv_weights_f8(w, C, 16, 1, 0)
    acc = ops.conv2d_nhwc_f8_acc(torch.from_numpy(np.ascontiguousarray(x)).cuda(), torch.from_numpy(packed).cuda(),
                                 256, 1, 1, 0)
    got = acc.cpu().numpy().reshape(256, 256)  # [pixel][oc]
    val = O.decode_f8(codes).astype(np.float64)
    exp = 64.0 * val[:, None] * val[None, :]
    bad = got != exp
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed("gpurun_out/f8_pair_probe.npz", got=got, exp=exp)
    print("pairs", got.size, "mismatching", int(bad.sum()), flush=True)
    if bad.any():
        i, j = np.nonzero(bad)
        for a, b in list(zip(i, j))[:20]:
            print(f"x=0x{codes[a]:02x} ({val[a]}) w=0x{codes[b]:02x} ({val[b]}): got {got[a, b]} exp {exp[a, b]}")


if __name__ == "__main__":
    main()
