"""bench.py's host-side choices (no GPU): the batch chooser."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_fit_batch_picks_the_largest_fitting_divisor():
    fit = _bench().fit_batch
    P, L = 25_000_000, 150
    GB = 1_000_000_000
    # one process (6 GB beside the pipeline) at the hg19 box's free HBM
    assert fit(12_500_000, P, L, int(92.5 * GB), headroom=6 << 30) == 12_500_000
    # torchrun (12 GB for the exchange): the next divisor of P
    assert fit(12_500_000, P, L, int(92.5 * GB), headroom=12 << 30) == 8_333_334
    assert fit(12_500_000, P, L, 60 * GB) == 6_250_000
    # never above the configured batch, never below the floor
    assert fit(6_250_000, P, L, 10_000 * GB) == 6_250_000
    assert fit(12_500_000, P, L, 0) >= 1_000_000
    # every choice is ceil(P / k): the batches of a step are equal but the last
    for free in (40, 70, 92, 100, 150):
        b = fit(12_500_000, P, L, free * GB)
        k = -(-P // b)
        assert b == -(-P // k)


def test_fit_batch_respects_the_library_batch_bound():
    """max_batch (smash_pipeline_max_batch: max_pairs * 2 * slots < 2^32)
    caps the batch even when the HBM would hold a larger one."""
    fit = _bench().fit_batch
    GB = 1_000_000_000
    P = 25_000_000
    mb = ((1 << 32) - 1) // (2 * 231)          # 250 bp mates
    b = fit(P, P, 250, 10_000 * GB, max_batch=mb)
    assert b <= mb and b == -(-P // -(-P // b))
    assert fit(12_500_000, P, 150, 10_000 * GB, max_batch=((1 << 32) - 1) // 262) == 12_500_000
