"""k_viterbi evaluates the transition cost |route/1000 - g|/beta with div1000() instead of
a division (reporter_amd/csrc/otr_kernels.h); this checks, over every u32 route length,
that it equals the IEEE quotient the oracle computes (oracle/oracle.c)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which('gcc') is None, reason='needs gcc')
def test_div1000_exhaustive(tmp_path):
    exe = str(tmp_path / 'div1000_check')
    # -mfma: the hardware fma (as v_fma_f64 on the GPU), not a libm emulation
    flags = ['-O2', '-ffp-contract=off']
    probe = subprocess.run(['gcc', '-mfma', '-E', '-x', 'c', '/dev/null'], capture_output=True)
    if probe.returncode == 0:
        flags.append('-mfma')
    subprocess.run(['gcc'] + flags + ['-o', exe, os.path.join(HERE, 'div1000_check.c'), '-lm'], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, check=True).stdout.strip()
    assert out == '0', 'div1000 differs from x / 1000.0 for %s inputs' % out
