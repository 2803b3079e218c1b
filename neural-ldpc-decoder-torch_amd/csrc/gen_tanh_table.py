"""Build the tanh correction table of the SP check node (lib/nldpc_tanh_ref.bin).

The reference's sum-product check node calls torch.tanh on a CPU fp32 tensor
(src/boosted_neural_ldpc_decoder/BoostedNeuralLDPCDecoder.py:402).  ATen evaluates it with the BLAS
vendor's vector math (this image's torch: MKL VML vsTanh, high-accuracy mode), whose results are
within one ulp of the correctly rounded tanh but not equal to it: 803 349 of the 1.09e9 fp32 inputs
with |x| <= 10 differ, by exactly one ulp (measured here; odd symmetric).  Through atanh's
1 / (1 - P^2) near saturation one ulp of a factor moves an SP message by up to ~1e-3 relative, so
the device reproduces torch.tanh exactly: it rounds a double-precision tanh (correct rounding except
near a halfway point) and applies this table of the inputs where torch.tanh differs.

The check-node inputs are -0.5 * clamp(m, -20, 20), so |x| <= 10 covers every value the decoder
evaluates.  Inputs whose double tanh lies within 8 double ulps of a fp32 halfway point are listed
separately with their exact torch.tanh value, so the table does not depend on which double tanh
the device uses.

File layout (little-endian uint32): magic 0x4841544E ("NTAH"), version 2, SH, KMAX, n_entries,
n_override; provenance[16] (64 bytes of NUL-padded ASCII: the torch version, ATen's CPU capability and
the CPU model of the build host -- the table is what THAT torch.tanh computes; tests compare it with
the torch of the machine they run on); idx[(KMAX >> SH) + 2] (bucket b = key >> SH holds entries idx[b]..idx[b+1]);
entries[n_entries] = key | dir << 31, ascending in key (key = |x| bits; dir 1: torch.tanh is one ulp
above the correctly rounded value, 0: one ulp below); overrides[n_override] = (key, result bits).

Usage: python3 gen_tanh_table.py OUT.bin
"""
import os
import struct
import sys

import numpy as np
import torch

SH = 15
KMAX = int(np.float32(10.0).view(np.uint32))  # 0x41200000


def provenance():
    """torch version | ATen CPU capability | CPU model of this host (what the table was measured on)."""
    cpu = "?"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "?")
    except OSError:
        pass
    return f"{torch.__version__}|{torch.backends.cpu.get_cpu_capability()}|{cpu}"


def main(out):
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    entries, overrides = [], []
    chunk = 1 << 24
    for base in range(0, KMAX + 1, chunk):
        u = np.arange(base, min(base + chunk, KMAX + 1), dtype=np.uint32)
        x = torch.from_numpy(u.view(np.float32))
        ref = torch.tanh(x).numpy().view(np.uint32)  # what the reference's torch computes
        d = torch.tanh(x.double())
        cr = d.float()
        # halfway point between cr and its neighbour on d's side
        crd = cr.double()
        nb = torch.nextafter(cr, torch.where(d > crd, torch.full_like(cr, 2.0), torch.full_like(cr, -2.0))).double()
        mid = 0.5 * (crd + nb)
        amb = ((d - mid).abs() <= 8 * d.abs() * 2.0 ** -52).numpy()
        crb = cr.numpy().view(np.uint32)
        diff = ref.astype(np.int64) - crb.astype(np.int64)
        if np.abs(diff[~amb]).max(initial=0) > 1:
            raise SystemExit("gen_tanh_table: torch.tanh is more than one ulp from the rounded double tanh")
        sel = (diff != 0) & ~amb
        entries.append(u[sel] | ((diff[sel] > 0).astype(np.uint32) << np.uint32(31)))
        for k in np.nonzero(amb)[0]:
            overrides.append((int(u[k]), int(ref[k])))
    ent = np.concatenate(entries).astype(np.uint32)
    keys = ent & np.uint32(0x7FFFFFFF)
    assert np.all(np.diff(keys.astype(np.int64)) > 0)
    nb = (KMAX >> SH) + 2
    idx = np.searchsorted(keys, (np.arange(nb, dtype=np.uint64) << np.uint64(SH)).astype(np.uint32)).astype(np.uint32)
    idx[-1] = len(ent)
    hdr = struct.pack("<6I", 0x4841544E, 2, SH, KMAX, len(ent), len(overrides)) + provenance().encode()[:63].ljust(64, b"\0")
    tmp = out + ".tmp"
    with open(tmp, "wb") as f:
        f.write(hdr)
        f.write(idx.tobytes())
        f.write(ent.tobytes())
        for k, v in overrides:
            f.write(struct.pack("<2I", k, v))
    os.replace(tmp, out)
    print(f"gen_tanh_table: {len(ent)} corrections, {len(overrides)} overrides -> {out}")


if __name__ == "__main__":
    main(sys.argv[1])
