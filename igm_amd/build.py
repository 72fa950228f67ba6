"""Build libigmhip.so (HIP, gfx950) in-tree and the CPU oracle (test infrastructure).

    python -m igm_amd.build            # both
    python -m igm_amd.build --lib      # libigmhip.so only

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the .so files travel to the GPU box with the repository snapshot.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, 'lib')
OBJDIR = os.path.join(ROOT, 'build', 'obj')
LIB = os.path.join(LIBDIR, 'libigmhip.so')
ARCH = os.environ.get('IGM_OFFLOAD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')

# per-translation-unit flags: the A-step restates NumPy/CPython arithmetic
# bit-for-bit, so it must not contract a*b+c into FMAs.
SOURCES = {
    'capi.hip': [],
    'actdist.hip': ['-ffp-contract=off'],
    # the f32 MD path uses the hardware sqrt/rcp (1-2 ulp); the f64 CG path is IEEE
    'mstep.hip': ['-fno-hip-fp32-correctly-rounded-divide-sqrt'],
    'hic_select.hip': ['-ffp-contract=off'],
    'violations.hip': ['-ffp-contract=off'],
    'asteps.hip': ['-ffp-contract=off'],
    'restraints.hip': ['-ffp-contract=off'],
}
# host-only C++ (no device code): the .hss / actdist.hdf5 reader and writer
HOST_SOURCES = {'h5io.cpp': []}
LIBS = ['-lz']
COMMON = ['-O3', '-fPIC', '-std=c++17', '--offload-arch=%s' % ARCH, '-Wall', '-Wno-unused-function',
          '-munsafe-fp-atomics', '-I%s' % os.path.join(ROOT, 'include')]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_lib(verbose=False):
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.h')]
    headers += [os.path.join(ROOT, 'include', h) for h in ('igm_hip.h', 'igm_io.h')]
    jobs = []
    objs = []
    for src, extra in SOURCES.items():
        sp = os.path.join(CSRC, src)
        if not os.path.exists(sp):
            continue
        op = os.path.join(OBJDIR, src.replace('.hip', '.o'))
        objs.append(op)
        if _newer(op, [sp] + headers):
            jobs.append([HIPCC] + COMMON + extra + ['-c', sp, '-o', op])
    for src, extra in HOST_SOURCES.items():
        sp = os.path.join(CSRC, src)
        op = os.path.join(OBJDIR, src.replace('.cpp', '.o'))
        objs.append(op)
        if _newer(op, [sp] + headers):
            jobs.append(['g++', '-O2', '-fPIC', '-std=c++17', '-Wall', '-Wextra', '-Wno-unused-parameter',
                         '-I%s' % os.path.join(ROOT, 'include')] + extra + ['-c', sp, '-o', op])

    def run(cmd):
        if verbose:
            print(' '.join(cmd), flush=True)
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError('hipcc failed:\n%s\n%s' % (' '.join(cmd), r.stdout))
        return r.stdout

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        for out in ex.map(run, jobs):
            if verbose and out.strip():
                print(out)
    if jobs or not os.path.exists(LIB):
        run([HIPCC, '--offload-arch=%s' % ARCH, '-shared', '-fPIC', '-o', LIB] + objs + LIBS)
    return LIB


def build_oracle(verbose=False):
    """The CPU oracle (tests / cpu_baseline only).  Also builds oracle/_ref from
    the reference's own C++ sources when /root/reference is present."""
    odir = os.path.join(ROOT, 'oracle')
    r = subprocess.run(['make', '-C', odir, '-j4'], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError('oracle build failed:\n' + r.stdout)
    if verbose:
        print(r.stdout)
    if os.path.isdir('/root/reference/igm/cython_compiled'):
        r = subprocess.run(['make', '-C', odir, 'ref'], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            raise RuntimeError('oracle/_ref build failed:\n' + r.stdout)
    return os.path.join(odir, 'liboracle.so')


if __name__ == '__main__':
    v = '-v' in sys.argv
    if '--oracle' not in sys.argv:
        print(build_lib(verbose=v))
    if '--lib' not in sys.argv:
        print(build_oracle(verbose=v))
