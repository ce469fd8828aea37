"""bench.py's byte model (CPU): per-stage algorithmic bytes for the forms the library
runs, and the check that flags a stage whose model would need more than the HBM
peak at its measured time (the old preprocess_bwd figure did)."""
import bench

C = dict(P=1_000_000, I=8_023_099, W=1920, H=1080, M=16)
S_C = 2_721_485  # row spans of config C's rect footprint (tools/span_stats.py)


def test_preprocess_bwd_model_is_below_peak_at_the_r05_time():
    # r05 driver line: preprocess_bwd 75.9 us; PMC-measured 397.7 MB per launch
    b = bench.algorithmic_bytes("preprocess_bwd", **C)
    assert b == 1_000_000 * (85 + 36 + 44 + 192)
    assert b <= 397.7e6 and b / 75.9e-6 / 1e9 < bench.HBM_PEAK_GBS
    # without a stored Jacobian (no backward prepared) the SH row is read instead
    assert bench.algorithmic_bytes("preprocess_bwd", **C, backward=False) == 1_000_000 * (85 + 192 + 44 + 192)
    # preprocess stores the Jacobian only when a backward follows
    assert (bench.algorithmic_bytes("preprocess", **C) - bench.algorithmic_bytes("preprocess", **C, backward=False)
            == 36 * 1_000_000)


def test_model_over_peak_flags_impossible_stages():
    per = {"preprocess_bwd": (0.0759, 100), "render_bwd": (0.2272, 100), "tile_sort": (0.0532, 100),
           "duplicate": (0.0207, 100), "scan": (0.025, 100)}
    fr = bench.stage_model_fracs(per, **C, S=S_C)
    assert set(fr) == set(per) and bench.model_over_peak(fr) == []
    # the r05 model of preprocess_bwd (P (92 + 147 + 24 M)) at the same time: 8.2 TB/s
    old = 1_000_000 * (92 + 147 + 24 * 16) / 75.9e-6 / 1e9 / bench.HBM_PEAK_GBS
    assert old > 1.0
    fast = dict(per, render_bwd=(0.01, 100))
    assert bench.model_over_peak(bench.stage_model_fracs(fast, **C, S=S_C)) == ["render_bwd"]


def test_rowspan_binning_model():
    P, I, W, H = C["P"], C["I"], C["W"], C["H"]
    T = 120 * 68
    assert bench.algorithmic_bytes("duplicate", **C, S=S_C) == P * 20 + S_C * 8
    assert bench.algorithmic_bytes("tile_sort", **C, S=S_C) == S_C * 12 + I * 4 + T * 8
    # the LSD sort's upstream-shaped figures without spans
    assert bench.algorithmic_bytes("tile_sort", **C) == I * 20 + T * 8
