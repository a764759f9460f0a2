"""Issue roofline of the search kernels from the SQ counter passes (tools/profile_sq.sh):
per launch, wave-instructions by unit against what the chip can issue in the launch's
cycles.  GRBM_GUI_ACTIVE counts shader cycles summed over the 8 XCDs; per CU (256) the
4 SIMDs retire one wave64 VALU instruction every 2 cycles each and the one scalar unit one
SALU instruction per cycle (MI355X_MICROARCH.md: VALU 2 cyc per wave64 op); LDS: one
instruction per CU per cycle at most.  frac = the busiest unit's share.
Usage: python tools/issue_roofline.py gpurun_out/sq5_c2dep KERNEL-SUBSTRING [...]"""
import json
import sys

sys.path.insert(0, __import__('os').path.dirname(__file__))
from sq_summary import main as _unused  # noqa: F401  (same directory layout)


def load(d):
    import subprocess
    out = subprocess.run([sys.executable, __file__.replace('issue_roofline.py', 'sq_summary.py'), d],
                         capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def roofline(k):
    cyc = k['GRBM_GUI_ACTIVE'] / 8.0  # shader cycles of the launch (per XCD)
    cus = 256
    valu = k['SQ_INSTS_VALU'] * 2.0 / (4 * cus * cyc)
    salu = k['SQ_INSTS_SALU'] / (cus * cyc)
    lds = k['SQ_INSTS_LDS'] / (cus * cyc)
    waves = k['SQ_WAVE_CYCLES'] / (4 * cus * cyc) * 4  # quad-cycles -> resident waves per SIMD
    return {'cycles': cyc, 'valu_insts': k['SQ_INSTS_VALU'], 'salu_insts': k['SQ_INSTS_SALU'],
            'lds_insts': k['SQ_INSTS_LDS'], 'vmem_rd': k['SQ_INSTS_VMEM_RD'], 'branch': k['SQ_INSTS_BRANCH'],
            'valu_issue_frac': round(valu, 3), 'salu_issue_frac': round(salu, 3), 'lds_issue_frac': round(lds, 3),
            'frac': round(max(valu, salu, lds), 3), 'bound': max((valu, 'VALU'), (salu, 'SALU'), (lds, 'LDS'))[1],
            'resident_waves_per_simd': round(waves, 2),
            'wait_share': round(k['SQ_WAIT_ANY'] / max(k['SQ_WAVE_CYCLES'], 1), 3)}


if __name__ == '__main__':
    d = load(sys.argv[1])
    out = {}
    for name, k in d.items():
        if any(s in name for s in sys.argv[2:]) and 'GRBM_GUI_ACTIVE' in k and 'SQ_INSTS_VALU' in k:
            out[name] = roofline(k)
    print(json.dumps(out, indent=1))
