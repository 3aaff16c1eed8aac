"""bench/run.py helpers that decide what a multi-GPU run measures (CPU)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_module():
    spec = importlib.util.spec_from_file_location("bench_run", os.path.join(ROOT, "bench", "run.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_transcode_batch_sizes_from_the_rank_share():
    """Config 3 at world 8 (256 pieces -> 32 per rank) must not run one half-padded batch: the
    batch is sized from the share so every rank pipelines >= 3 equal batches."""
    tb = _run_module().transcode_batch
    for world in (1, 2, 4, 8):
        n = 256 // world
        b = tb(n, 64)
        assert n % b == 0 and n // b >= 3 and b <= 64, (world, b)
    assert tb(256, 64) == 64 and tb(32, 64) == 8
    assert tb(2, 64) == 2 and tb(1, 64) == 1        # fewer pieces than batches: one full batch
    assert tb(33, 64) == 11                          # an odd share still divides evenly
