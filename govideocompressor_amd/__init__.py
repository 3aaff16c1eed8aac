"""govideocompressor_amd -- MI355X-native distributed video compressor.

Same capabilities as GPUs/goVideoCompressor (split -> pull-scheduled segment
transcoding -> ordered merge, with the `server s|c|t` / worker job API), but the
codec runs as hand-written gfx950 HIP kernels on PyTorch-ROCm tensors and the
intra-node data plane is RCCL over xGMI.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
