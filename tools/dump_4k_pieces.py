"""Write a few 4K30 input pieces (the config-3 bench's inputs: GPU H.264 CRF 20 and GPU HEVC
CRF 22 encodes of synth_clip content) to gpurun_out/pieces/, for profiling the host parse
on the CPU.  Run on an MI355X: ``python tools/dump_4k_pieces.py [n]``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from govideocompressor_amd.models.h264_gpu import GpuH264Encoder, H264Params, synth_clip
    from govideocompressor_amd.models.hevc_gpu import GpuHevcEncoder, HevcParams
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    W, H, F = 3840, 2160, 30
    out = os.path.join("gpurun_out", "pieces")
    os.makedirs(out, exist_ok=True)
    y, u, v = synth_clip(n, F, W, H, seed=3)
    for codec, enc in (("264", GpuH264Encoder(H264Params(width=W, height=H, crf=20), slots=n)),
                       ("265", GpuHevcEncoder(HevcParams(width=W, height=H, crf=22.0), slots=n))):
        for i, r in enumerate(enc.encode(y, u, v, metrics=False)):
            with open(os.path.join(out, f"p{i}.{codec}"), "wb") as f:
                f.write(r.bitstream)
        enc.close()
    print("wrote", sorted(os.listdir(out)))


if __name__ == "__main__":
    main()
