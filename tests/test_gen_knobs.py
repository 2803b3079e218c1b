"""Every generator knob left after the r5 prune (csrc/gen_fused.py: NLDPC_GEN_*) still generates and compiles:
one built-in geometry (BG2 z=16), each non-default knob setting, hipcc --genco for gfx950 (CPU only).  The
default kernels are the library's own build and the GPU suite's subject; this covers the settings no GPU run
loads (experiment and diagnostic builds)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

from conftest import ROOT

CS = os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# (name, environment, translation units to compile)
VARIANTS = [
    ("wlate_all", {"NLDPC_GEN_WLATE": "1"}, ["fused_bg2_z16_s0.hip"]),
    ("wlate_none", {"NLDPC_GEN_WLATE": "0", "NLDPC_GEN_KINDS": "1"}, ["fused_bg2_z16_s2.hip"]),
    ("stamps", {"NLDPC_GEN_STAMPS": "1", "NLDPC_GEN_NOBWD": "1"}, ["fused_bg2_z16_s0.hip", "fused_bg2_z16_s1.hip"]),
    ("geom", {"NLDPC_GEN_GEOM": "bg2_z16:8,2,1"}, ["fused_bg2_z16_s0.hip", "fused_bg2_z16_bwd.hip"]),
    ("skip", {"NLDPC_GEN_SKIP": "sync,cnmath,d1post,wload,cnread,cnwrite"}, ["fused_bg2_z16_s3.hip"]),
    ("parts", {"NLDPC_GEN_PARTS": "1"}, ["fused_bg2_z16_s0.hip"]),
    # (r6 backward defaults off: the r5 read-backs and check node)
    ("bwd_r5", {"NLDPC_GEN_BWDPIPE": "0", "NLDPC_GEN_CNBSPARSE": "0", "NLDPC_GEN_KINDS": "2"}, ["fused_bg2_z16_bwd.hip"]),
    ("cache_r5", {"NLDPC_GEN_BWDCACHE": "0", "NLDPC_GEN_FWDNT8": "0", "NLDPC_GEN_KINDS": "2"},
     ["fused_bg2_z16_bwd.hip", "fused_bg2_z16_s1.hip"]),
    # (fetch bisect of the training forward, r6: the posteriors' channel re-reads replaced by registers)
    ("skip_xl", {"NLDPC_GEN_SKIP": "xlreg,xld1", "NLDPC_GEN_KINDS": "2", "NLDPC_GEN_NOBWD": "1"}, ["fused_bg2_z16_s1.hip"]),
    # (r6: the MODE-6 decode -- UCN with CN / UCN / VN weights compiled in -- for another graph than the default's)
    ("ucnw_z16", {"NLDPC_GEN_UCNW": "bg2_z16", "NLDPC_GEN_KINDS": "1", "NLDPC_GEN_NOBWD": "1"}, ["fused_bg2_z16_s0u.hip"]),
    # (UREMAT applies to one-codeword geometries: BG2 z=384's training forward; z=16 packs 16 codewords)
    ("uremat_off", {"NLDPC_GEN_UREMAT": "0", "NLDPC_GEN_ONLY": "bg2_z384", "NLDPC_GEN_KINDS": "3",
                    "NLDPC_GEN_NOBWD": "1"}, ["fused_bg2_z384_s1.hip"]),
]


def _build(tmp, name, env, units):
    out = os.path.join(tmp, name)
    e = dict(os.environ, NLDPC_GEN_ONLY="bg2_z16", NLDPC_GEN_KINDS="3")
    e.update(env)
    subprocess.run([sys.executable, os.path.join(CS, "gen_fused.py"), out, os.path.join(ROOT, "resources")],
                   env=e, check=True, capture_output=True)
    for u in units:
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "--genco", "-O1", "-std=c++17", "-ffp-contract=off",
                            "-I" + os.path.join(ROOT, "include"), "-I" + CS, "-x", "hip",
                            os.path.join(out, u), "-o", os.path.join(out, u + ".co")], capture_output=True, text=True)
        if r.returncode != 0:
            return f"{name}/{u}: {r.stderr[-2000:]}"
        if os.path.getsize(os.path.join(out, u + ".co")) < 1000:
            return f"{name}/{u}: empty code object"
    return None


def test_every_knob_generates_and_compiles(tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        errs = [r for r in ex.map(lambda v: _build(str(tmp_path), *v), VARIANTS) if r]
    assert not errs, "\n".join(errs)


def test_no_pruned_knob_is_read():
    """The generator reads only the knobs this file lists (the r5 prune): no measured loser comes back as
    an untested branch."""
    import re
    src = open(os.path.join(CS, "gen_fused.py")).read()
    knobs = set(re.findall(r'environ\.get\("(NLDPC_[A-Z_0-9]+)"', src))
    assert knobs <= {"NLDPC_GEN_PARTS", "NLDPC_GEN_SKIP", "NLDPC_GEN_STAMPS", "NLDPC_GEN_GEOM", "NLDPC_GEN_WLATE",
                     "NLDPC_GEN_NOBWD", "NLDPC_GEN_ONLY", "NLDPC_GEN_KINDS", "NLDPC_FUSED_EXTRA", "NLDPC_GEN_UREMAT",
                     "NLDPC_GEN_BWDPIPE", "NLDPC_GEN_CNBSPARSE", "NLDPC_GEN_BWDCACHE", "NLDPC_GEN_FWDNT8",
                     "NLDPC_GEN_UCNW"}, knobs
    assert len(knobs) <= 15
