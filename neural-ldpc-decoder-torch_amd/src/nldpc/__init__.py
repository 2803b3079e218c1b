"""MI355X-native neural belief-propagation LDPC decoding (host runtime).

Layers:
  nldpc._lib        ctypes binding of libnldpc.so (include/nldpc.h): HIP kernels for gfx950
  nldpc.graph       lifted QC graph as an edge list, device handles
  nldpc.decode      decode / autograd over nldpc_forward / nldpc_backward
  nldpc.channel     on-device AWGN channel and fused BER/FER counters
  nldpc.distributed one-process-per-GPU sharded decoding with an RCCL reduction of the counters
The drop-in packages neural_ldpc_decoder, boosted_neural_ldpc_decoder and checkpoint_utils (next to
this package) mirror the reference's Python API on top of it.
"""
from .graph import LiftedGraph  # noqa: F401
from .decode import DecodeCfg, decode, decode_autograd, KIND_SP, KIND_MS, KIND_QMS, KIND_NEURAL  # noqa: F401
