"""GPU A/B helper: one cfg5 training step (BoostedNeuralLDPCDecoder QMS q=5 NW(3,0,3), BG2 z=384, T=50; forward +
LDPCDecoderLoss BCE + backward, no optimizer step) on the library NLDPC_LIB_PATH names, and a digest of the loss and
every parameter gradient -- two libraries whose backward kernels differ only in form print the same line iff their
gradients are bit-identical.  Usage: NLDPC_LIB_PATH=... python tools/grad_digest.py [B]"""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "neural-ldpc-decoder-torch_amd", "src"), ROOT]

from boosted_neural_ldpc_decoder.BoostedNeuralLDPCDecoder import BoostedNeuralLDPCDecoder  # noqa: E402
from boosted_neural_ldpc_decoder.ConnectingMatrix import ConnectingMatrix  # noqa: E402
from boosted_neural_ldpc_decoder.ConnectingMatrixTorch import ConnectingMatrixTorch  # noqa: E402
from boosted_neural_ldpc_decoder.LDPCDecoderLoss import LDPCDecoderLoss  # noqa: E402
from boosted_neural_ldpc_decoder.struct.DecoderType import DecoderType  # noqa: E402
from boosted_neural_ldpc_decoder.struct.LossType import LossType  # noqa: E402
from boosted_neural_ldpc_decoder.struct.NodeWeightSharingConfig import NodeWeightSharingConfig  # noqa: E402
from nldpc.channel import awgn_llr, boosted_code_rate, sigma_for  # noqa: E402

B, T, Z = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 50, 384
dev = torch.device("cuda", 0)
bg = np.loadtxt(os.path.join(ROOT, "resources", "basegraph2_set0.txt"), int, delimiter="\t")
M, N = bg.shape
conn = ConnectingMatrixTorch(ConnectingMatrix(Z, bg), device=dev)
model = BoostedNeuralLDPCDecoder(T, B, conn, node_weight_sharing_config=NodeWeightSharingConfig(3, 0, 3),
                                 decoding_type=DecoderType.QMS, decoder_qms_qbit=5).to(dev)
g = torch.Generator().manual_seed(11)
with torch.no_grad():  # weights off their 1.0 init, so every mask and product is exercised
    for p in model.parameters():
        p.copy_((0.6 + 0.8 * torch.rand(p.shape, generator=g)).to(dev))
xa = awgn_llr(B, N, Z, sigma_for(1.5, boosted_code_rate(N, M)), seed=2042, qbit=5, device=dev)
y = torch.zeros(B, N * Z, device=dev)
model.train()
outs = model(xa, target_iter=list(range(T)))
loss = LDPCDecoderLoss(loss_type=LossType.BCE, etha=1.0)(outs, y, coeff_param=list(range(T)))
loss.backward()
h = hashlib.sha256()
h.update(np.float64(loss.item()).tobytes())
n = 0
for name, p in sorted(model.named_parameters()):
    if p.grad is not None:
        h.update(name.encode())
        h.update(p.grad.detach().cpu().numpy().tobytes())
        n += 1
print(f"loss {loss.item():.9g}  grads {n}  digest {h.hexdigest()[:32]}")
