"""div_by_rcp (csrc/dpath.h), the axis-aligned scan groups' quotient: a * RN(1/b)
with two FMA residual corrections must equal IEEE a / b bit for bit over the range
scan_pair admits it for (|b| >= 2^-60, quotients >= 2^-31 in magnitude).  Runs
tools/gpu_runs/r05/fast_div_check.c (the host restatement, x86 FMA) on a few million random
and edge-mantissa pairs; the round-5 run covered 1.6e9."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fast_division_matches_ieee(tmp_path):
    exe = tmp_path / 'fdc'
    subprocess.run(['gcc', '-O2', '-ffp-contract=off', '-mfma', '-o', str(exe),
                    os.path.join(REPO, 'tools', 'gpu_runs', 'r05', 'fast_div_check.c'), '-lm'], check=True)
    out = subprocess.run([str(exe), '4000000'], check=True, capture_output=True, text=True).stdout
    last = out.strip().splitlines()[-1].split()
    assert last[0] == 'checked' and int(last[1]) > 3_000_000
    assert last[2] == 'bad' and int(last[3]) == 0, out
