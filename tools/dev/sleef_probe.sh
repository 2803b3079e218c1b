# Builds and runs the exhaustive SLEEF restatement check on the CPU (development container).
set -e
D=$(cd "$(dirname "$0")" && pwd); R=$D/../..
TL=$(python3 -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
g++ -O2 -std=c++17 -mavx512f -mfma -ffp-contract=off -I$R/neural-ldpc-decoder-torch_amd/csrc $D/sleef_probe.cpp \
    -L$TL -ltorch_cpu -lc10 -Wl,-rpath,$TL -o /tmp/sleef_probe
time /tmp/sleef_probe
