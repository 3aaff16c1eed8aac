"""Codec "model families".  ``h264_gpu``: the gfx950 H.264 encoder; ``h264_cpu``:
the CPU reference backend; see :func:`govideocompressor_amd.models.registry.get_backend`."""
