"""Build the native libraries in-tree (lib/*.so travel to the GPU box with the snapshot).

* lib/libbls381.so            -- the product: hipcc --offload-arch=gfx950, C ABI of include/bls381.h
* lib/libbls381_hostcheck.so  -- test infrastructure: g++ build of the same arithmetic headers
* tools/valu_peak             -- integer-VALU peak microbenchmark (roofline denominator)
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
INC = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_SOURCES = ["bls381_capi.hip"]
HEADERS = ["bls381_defs.hpp", "bls381_consts.hpp", "bls381_field.hpp", "bls381_curve.hpp", "bls381_hash.hpp",
           "bls381_lazy.hpp", "bls381_pairing.hpp", "bls381_pair.hpp", "bls381_quad.hpp", "bls381_ssz.hpp",
           "bls381_kernels.hpp"]


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _run(cmd):
    print("+", " ".join(cmd), file=sys.stderr, flush=True)
    subprocess.run(cmd, check=True)


def build_hip(force=False, extra=(), out=None):
    """out: another target (a measurement variant, variants/<name>/libbls381.so, built with `extra`
    defines and selected at run time through BLS381_LIB)."""
    os.makedirs(LIB, exist_ok=True)
    out = out or os.path.join(LIB, "libbls381.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    deps = [os.path.join(CSRC, f) for f in HIP_SOURCES + HEADERS] + [os.path.join(INC, "bls381.h")]
    if not force and _newer(out, deps):
        return out
    import fcntl
    import shutil
    import tempfile
    # one build of a target at a time (a second builder waits, then finds it current)
    with open(out + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and _newer(out, deps):
            return out
        # built beside the target under a name of its own and renamed into place, so a snapshot of
        # the tree taken while hipcc runs (a GPU call) sees the old library or the new one, never a
        # partial file
        fd, tmp = tempfile.mkstemp(prefix=os.path.basename(out) + ".", suffix=".partial", dir=os.path.dirname(out))
        os.close(fd)
        # the newest source mtime at the start: the library is stamped with it, so a source edited
        # during the build stays newer (rebuilt next time) and an unchanged tree stays current
        src_t = max(os.path.getmtime(d) for d in deps)
        try:
            # hipcc reads the sources twice (device code, then host code, minutes apart): it compiles
            # a snapshot, so an edit during the build can never pair one version's kernels with
            # another's launch code (a kernel symbol the code object lacks)
            with tempfile.TemporaryDirectory(prefix="bls381_build_") as snap:
                shutil.copytree(CSRC, os.path.join(snap, "csrc"))
                shutil.copytree(INC, os.path.join(snap, "include"))
                scs = os.path.join(snap, "csrc")
                _run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-I",
                      os.path.join(snap, "include"), "-I", scs, *extra, *[os.path.join(scs, f) for f in HIP_SOURCES],
                      "-o", tmp])
            os.chmod(tmp, 0o755)
            os.replace(tmp, out)
        finally:
            if os.path.exists(tmp):
                os.unlink(tmp)
        os.utime(out, (src_t, src_t))
    return out


# the ASan/UBSan host build (~60 MB) is a CPU-test artefact: it lives outside the tree,
# so it never rides along to the GPU box
SANITIZE_DIR = os.environ.get("BLS381_SANITIZE_DIR", os.path.expanduser("~/.cache/bls381_amd"))


def build_hostcheck(force=False, sanitize=False, count_ops=False, defines=()):
    """defines: build-knob variants (e.g. ("BLS_WAVES_PER_EU=1",)) -- test-only, built out of
    tree like the sanitized library."""
    os.makedirs(LIB, exist_ok=True)
    name = "libbls381_hostcheck_asan.so" if sanitize else (
        "libbls381_hostcheck_count.so" if count_ops else "libbls381_hostcheck.so")
    if defines:
        name = name[:-3] + "_" + "_".join(d.replace("=", "").lower() for d in defines) + ".so"
    if sanitize or defines:
        os.makedirs(SANITIZE_DIR, exist_ok=True)
    out = os.path.join(SANITIZE_DIR if (sanitize or defines) else LIB, name)
    src = os.path.join(CSRC, "host_check.cpp")
    deps = [src] + [os.path.join(CSRC, f) for f in HEADERS if f != "bls381_kernels.hpp"]
    if not force and _newer(out, deps):
        return out
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-pthread", "-Wall", "-Wno-unknown-pragmas", "-I", CSRC, src, "-o", out]
    if sanitize:
        # -O0: the sanitized build of these fully unrolled headers takes ~10 min at -O2 -g
        cmd[2:3] = ["-O0", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    if count_ops:
        cmd[3:3] = ["-DBLS_COUNT_OPS"]
    cmd[3:3] = ["-D" + d for d in defines]
    _run(cmd)
    return out


def build_valu_peak(force=False):
    src = os.path.join(ROOT, "tools", "valu_peak.hip")
    out = os.path.join(ROOT, "tools", "valu_peak")
    if not force and _newer(out, [src]):
        return out
    _run([HIPCC, "--offload-arch=gfx950", "-O3", src, "-o", out])
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    build_hostcheck(force)
    build_hostcheck(force, count_ops=True)
    build_valu_peak(force)
    build_hip(force)
