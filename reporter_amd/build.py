"""Builds every native artefact in-tree (no JIT cache, so the .so files travel to the GPU box).

  reporter_amd/libotr.so            product: HIP kernels (gfx950) + C-ABI (include/otr.h)
  reporter_amd/tools/libotrgen.so   workload generator (bench/test infrastructure)
  oracle/liboracle.so               CPU oracle (test infrastructure, plain C)

libotr.so links the HIP runtime that ships with the installed PyTorch when there is
one, so that a Python process using torch.distributed and libotr shares ONE HIP
runtime (two copies in one process would each own the device).
"""
import importlib.util
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'reporter_amd')
CSRC = os.path.join(PKG, 'csrc')
BUILD = os.path.join(ROOT, 'build', 'obj')
ARCH = os.environ.get('OTR_OFFLOAD_ARCH', 'gfx950')
HIPCC = shutil.which('hipcc') or '/opt/rocm/bin/hipcc'

HIP_FLAGS = ['--offload-arch=' + ARCH, '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off', '-fno-fast-math',
             '-Wall', '-Wno-unused-function', '-Wno-unused-variable', '-Wno-unused-but-set-variable',
             '-I' + os.path.join(ROOT, 'include')]


def source_hash():
    """Identity of the libotr.so sources (the HIP/C++ sources, headers and compile flags):
    a PMC summary recorded from one build is attached to bench lines of that build only."""
    import hashlib
    # (the flags without the include path: the same sources built in another checkout —
    # the GPU box's copy, /root/repo or its symlink target — are the same build)
    h = hashlib.sha1(' '.join(f for f in HIP_FLAGS[1:] if not f.startswith('-I')).encode())
    for d in (CSRC, os.path.join(ROOT, 'include')):
        for f in sorted(os.listdir(d)):
            if f.endswith(('.h', '.hip', '.cpp')):
                h.update(f.encode())
                with open(os.path.join(d, f), 'rb') as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


def hip_runtime_dir():
    spec = importlib.util.find_spec('torch')
    if spec and spec.origin:
        d = os.path.join(os.path.dirname(spec.origin), 'lib')
        if os.path.exists(os.path.join(d, 'libamdhip64.so')):
            return d, 'libamdhip64.so'
    return '/opt/rocm/lib', 'libamdhip64.so.7'


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError('build step failed: ' + ' '.join(cmd))
    return r.stdout


def _newer(target, sources):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


def build_otr(force=False, stamps=False, variant=None, defines=()):
    """stamps=True: diagnostic build with per-phase shader-clock stamps (libotr_stamps.so).
    variant/defines: an A/B build libotr_<variant>.so with extra -D flags (experiments)."""
    os.makedirs(BUILD, exist_ok=True)
    suffix = '_stamps' if stamps else ''
    extra = ['-DOTR_STAMPS'] if stamps else []
    if variant:
        suffix += '_' + variant
        extra += ['-D' + d for d in defines]
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')]
    headers += [os.path.join(ROOT, 'include', f) for f in os.listdir(os.path.join(ROOT, 'include'))]
    objs, jobs = [], []
    for src in ('otr_engine.hip', 'otr_api.cpp', 'otr_service.cpp', 'otr_graph_build.cpp'):
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src + suffix + '.o')
        objs.append(o)
        if force or not _newer(o, [s] + headers):
            lang = [] if src.endswith('.hip') else ['-x', 'hip']
            jobs.append([HIPCC] + HIP_FLAGS + extra + lang + ['-c', s, '-o', o])
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(_run, jobs))
    lib = os.path.join(PKG, 'libotr%s.so' % suffix)
    if force or not _newer(lib, objs):
        rdir, rname = hip_runtime_dir()
        _run(['g++', '-shared', '-o', lib] + objs +
             ['-L' + rdir, '-l:' + rname, '-Wl,-rpath,' + rdir, '-Wl,--no-undefined', '-lpthread'])
    return lib


def build_gen(force=False):
    src = os.path.join(PKG, 'tools', 'otrgen.cpp')
    lib = os.path.join(PKG, 'tools', 'libotrgen.so')
    if force or not _newer(lib, [src, os.path.join(ROOT, 'include', 'otr_graph_format.h')]):
        _run(['g++', '-O2', '-std=c++17', '-fPIC', '-shared', '-o', lib, src])
    return lib


def build_oracle(force=False):
    args = ['make', '-C', os.path.join(ROOT, 'oracle')]
    if force:
        args += ['-B']
    _run(args)
    return os.path.join(ROOT, 'oracle', 'liboracle.so')


def build_calib(force=False):
    """tools/calib_fetch: known-byte access shapes for calibrating FETCH_SIZE/WRITE_SIZE
    (profiling infrastructure, run by tools/profile_gpu.sh)."""
    src = os.path.join(PKG, 'tools', 'calib_fetch.hip')
    exe = os.path.join(PKG, 'tools', 'calib_fetch')
    if force or not _newer(exe, [src]):
        rdir, rname = hip_runtime_dir()
        _run([HIPCC] + HIP_FLAGS + ['-o', exe, src, '-Wl,-rpath,' + rdir])
    return exe


def build_loadgen(force=False):
    """tools/loadgen: concurrent otr_report callers with/without the coalescer (bench tool)."""
    src = os.path.join(PKG, 'tools', 'loadgen.cpp')
    exe = os.path.join(PKG, 'tools', 'loadgen')
    lib = os.path.join(PKG, 'libotr.so')
    if force or not _newer(exe, [src, lib, os.path.join(ROOT, 'include', 'otr.h')]):
        _run(['g++', '-O2', '-g', '-rdynamic', '-std=c++17', '-o', exe, src, '-L' + PKG, '-l:libotr.so',
              '-Wl,-rpath,' + PKG, '-lpthread'])
    return exe


def build_parsecheck(force=False):
    """tools/libparsecheck.so: host build of the ingest number parsers (CPU tests only)."""
    src = os.path.join(PKG, 'tools', 'parsecheck.cpp')
    lib = os.path.join(PKG, 'tools', 'libparsecheck.so')
    deps = [src] + [os.path.join(CSRC, f) for f in ('otr_ingest.h', 'otr_pow5.h')]
    if force or not _newer(lib, deps):
        _run([HIPCC, '-x', 'hip', '--cuda-host-only', '-O2', '-std=c++17', '-fPIC', '-shared',
              '-I' + os.path.join(ROOT, 'include'), '-o', lib, src])
    return lib


def build_mincheck(force=False):
    """tools/libmincheck.so: host build of the node tables' IN-gap codes (CPU tests only)."""
    src = os.path.join(PKG, 'tools', 'mincheck.cpp')
    lib = os.path.join(PKG, 'tools', 'libmincheck.so')
    deps = [src, os.path.join(CSRC, 'otr_mincode.h')]
    if force or not _newer(lib, deps):
        _run([HIPCC, '-x', 'hip', '--cuda-host-only', '-O2', '-std=c++17', '-fPIC', '-shared', '-o', lib, src])
    return lib


def build_all(force=False):
    """Everything, the three libotr builds in parallel (each compiles its HIP sources for
    gfx950).  force=True recompiles every object (what the driver's build() does)."""
    from concurrent.futures import ThreadPoolExecutor
    build_gen(force)
    build_parsecheck(force)
    build_mincheck(force)
    build_oracle(force)
    build_calib(force)
    with ThreadPoolExecutor(max_workers=3) as ex:
        futs = [ex.submit(build_otr, force),
                # test build: every first-tier search goes down the retry tiers (tests/test_gpu_tiers.py)
                # (and every node retry tier resumes / dumps: OTR_ND_IN_MIN / OTR_ND_OUT_MIN 0;
                # short pending lists in the 1024- / 2048-slot and the first edge-state tables,
                # so searches whose frontier outgrows them take the restart path)
                ex.submit(build_otr, force, False, 'tiercheck', ['OTR_FORCE_RETRY', 'OTR_ND_IN_MIN=0',
                                                                 'OTR_ND_OUT_MIN=0', 'OTR_PCAP1024=96',
                                                                 'OTR_PCAP2048=160', 'OTR_E1PCAP=64']),
                # test build: every search in the global-memory kernel (tests/test_gpu_tiers.py)
                ex.submit(build_otr, force, False, 'generalcheck', ['OTR_FORCE_GENERAL'])]
        lib = futs[0].result()
        for f in futs[1:]:
            f.result()
    build_loadgen(force)
    return lib


if __name__ == '__main__':
    if '--variant' in sys.argv:  # --variant NAME DEF1 DEF2 ...
        i = sys.argv.index('--variant')
        print(build_otr(force=True, stamps='--stamps' in sys.argv, variant=sys.argv[i + 1],
                        defines=[d for d in sys.argv[i + 2:] if not d.startswith('--')]))
    elif '--stamps' in sys.argv:
        print(build_otr(force='--force' in sys.argv, stamps=True))
    else:
        print(build_all(force='--force' in sys.argv))
