"""govideocompressor_amd -- MI355X-native distributed video compressor.

Same capabilities as GPUs/goVideoCompressor (split -> pull-scheduled segment
transcoding -> ordered merge, with the `server s|c|t` / worker job API), but the
codec runs as hand-written gfx950 HIP kernels on PyTorch-ROCm tensors and the
intra-node data plane is RCCL over xGMI.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"

import os as _os

# The encoder keeps up to seven HIP streams busy at once (compute, CABAC binarisation,
# arithmetic coding, the merge, the next batch's synthesis / decode and lookahead).  With HIP's
# default of 4 hardware queues, streams share queues round-robin, and a 200 ms arithmetic-coding
# launch then blocks the binarisation kernels the compute stream waits on (round-4 trace: the
# compute stream idle for the whole coder launch, 250 ms per 256 x 60-frame batch).
# A value below 8 is raised (the GPU boxes export HIP's default of 4; round-4 trace: the coder
# and the binariser still shared a queue with the default only).  It has to be in the
# environment before the HIP runtime initialises.
try:
    if int(_os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
        _os.environ["GPU_MAX_HW_QUEUES"] = "8"
except ValueError:
    _os.environ["GPU_MAX_HW_QUEUES"] = "8"
