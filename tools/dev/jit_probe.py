"""Probe (development only, r3): after this process has initialised the GPU, can it (1) run hipcc as a
child process and load the code object it writes, (2) compile with hiprtc in-process?"""
import ctypes
import os
import subprocess
import sys
import tempfile
import time

import torch

x = torch.ones(4, device="cuda")  # the GPU is initialised from here on
src = 'extern "C" __global__ void k(float* p) { p[threadIdx.x] *= 2.f; }\n'
d = tempfile.mkdtemp()
open(os.path.join(d, "k.hip"), "w").write(src)
t0 = time.time()
r = subprocess.run(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O3", os.path.join(d, "k.hip"), "-o",
                    os.path.join(d, "k.co")], capture_output=True, text=True)
print("hipcc child after GPU init: rc", r.returncode, "in %.1f s" % (time.time() - t0), r.stderr[-300:])
hip = ctypes.CDLL("libamdhip64.so")
mod = ctypes.c_void_p()
fn = ctypes.c_void_p()
if r.returncode == 0:
    data = open(os.path.join(d, "k.co"), "rb").read()
    e1 = hip.hipModuleLoadData(ctypes.byref(mod), data)
    e2 = hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"k")
    p = ctypes.c_void_p(x.data_ptr())
    args = (ctypes.c_void_p * 1)(ctypes.addressof(p))
    e3 = hip.hipModuleLaunchKernel(fn, 1, 1, 1, 4, 1, 1, 0, None, args, None)
    torch.cuda.synchronize()
    print("module load/get/launch:", e1, e2, e3, x.tolist())
try:
    rtc = ctypes.CDLL("libhiprtc.so")
    prog = ctypes.c_void_p()
    print("hiprtcCreateProgram", rtc.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"k.hip", 0, None, None))
    opts = (ctypes.c_char_p * 2)(b"--offload-arch=gfx950", b"-O3")
    t0 = time.time()
    print("hiprtcCompileProgram", rtc.hiprtcCompileProgram(prog, 2, opts), "in %.1f s" % (time.time() - t0))
except OSError as e:
    print("hiprtc:", e)
sys.stdout.flush()
