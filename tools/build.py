"""Build every native artefact in-tree (used by __graft_entry__.build()).

  unipeak_amd/lib/libunipeak_hip.so   HIP kernels + C-ABI (gfx950)
  bin/regions, bin/strand_shift, bin/tags_in_regions, bin/convert_align
                                      C++ host CLIs
  oracle/_build/liboracle.so, oracle/_build/orc        CPU restatement
                                                       (test infrastructure)
Rebuilds only what is older than its sources.
"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("UNIPEAK_ARCH", "gfx950")


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _includes(src, seen=None):
    """src and the files it #includes with quotes, recursively (from its
    own directory or include/)"""
    import re
    seen = set() if seen is None else seen
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    for m in re.finditer(r'^\s*#\s*include\s+"([^"]+)"', open(src, errors="replace").read(), re.M):
        for d in (os.path.dirname(src), os.path.join(ROOT, "include")):
            f = os.path.join(d, m.group(1))
            if os.path.exists(f):
                _includes(f, seen)
                break
    return seen


def _run(cmd, cwd=ROOT):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


def compile_lib(out, extra=(), jobs=None):
    """libunipeak_hip.so from six translation units compiled in parallel:
    api.hip (C-ABI, non-templated kernels), tir.hip (tags_in_regions) and
    nh_tu.hip once per window width NH = 1..8 (the templated K1/K3/K4
    kernels)."""
    from concurrent.futures import ThreadPoolExecutor
    csrc = os.path.join(ROOT, "unipeak_amd", "csrc")
    objdir = os.path.join(ROOT, "build", "obj_" + os.path.basename(out).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
             "-I", os.path.join(ROOT, "include")] + list(extra)
    units = [("api", os.path.join(csrc, "api.hip"), []),
             ("tir", os.path.join(csrc, "tir.hip"), []),
             ("countmap", os.path.join(csrc, "countmap.hip"), [])] + [
        (f"nh{k}", os.path.join(csrc, "nh_tu.hip"), [f"-DUPK_NH_TU={k}"]) for k in range(1, 9)]
    stamp = os.path.join(objdir, "flags.txt")  # objects built with other flags are stale
    same = os.path.exists(stamp) and open(stamp).read() == " ".join(flags)
    if not same and os.path.exists(stamp):
        os.remove(stamp)  # a partial build with new flags must not inherit the old stamp
    def one(u):
        name, src, defs = u
        obj = os.path.join(objdir, name + ".o")
        if not same or _stale(obj, _includes(src)):
            _run([HIPCC] + flags + defs + ["-c", "-o", obj, src])
        return obj
    with ThreadPoolExecutor(jobs or min(7, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(one, units))
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    with open(stamp, "w") as f:  # only after every object and the link succeeded
        f.write(" ".join(flags))
    return out


def build_lib(force=False):
    out = os.path.join(ROOT, "unipeak_amd", "lib", "libunipeak_hip.so")
    srcs = glob.glob(os.path.join(ROOT, "unipeak_amd", "csrc", "*")) + [
        os.path.join(ROOT, "include", "unipeak_hip.h")]
    if force or _stale(out, srcs):
        compile_lib(out)
    return out


def build_cli(force=False):
    lib = os.path.join(ROOT, "unipeak_amd", "lib")
    hsrc = sorted(glob.glob(os.path.join(ROOT, "unipeak_amd", "host", "*.cpp")))
    hdrs = glob.glob(os.path.join(ROOT, "unipeak_amd", "host", "*.hpp"))
    if not hsrc:
        return []
    common = [s for s in hsrc if not os.path.basename(s).startswith("main_")]
    outs = []
    os.makedirs(os.path.join(ROOT, "bin"), exist_ok=True)
    for m in [s for s in hsrc if os.path.basename(s).startswith("main_")]:
        name = os.path.basename(m)[len("main_"):-len(".cpp")]
        out = os.path.join(ROOT, "bin", name)
        deps = common + hdrs + [m, os.path.join(lib, "libunipeak_hip.so"),
                                os.path.join(ROOT, "include", "unipeak_hip.h")]
        if force or _stale(out, deps):
            _run(["g++", "-O2", "-std=c++17", "-Wall", "-ffp-contract=off", "-fno-fast-math",
                  "-I", os.path.join(ROOT, "include"), "-o", out, m] + common +
                 ["-L", lib, "-lunipeak_hip", "-Wl,-rpath,$ORIGIN/../unipeak_amd/lib",
                  "-lpthread", "-lz"])
        outs.append(out)
    return outs


def build_oracle(force=False):
    if force:
        _run(["make", "-C", os.path.join(ROOT, "oracle"), "clean"])
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def build_all(force=False):
    build_oracle(force)
    build_lib(force)
    build_cli(force)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":  # tools/build.py --variant NAME -DFLAG ...
        compile_lib(os.path.join(ROOT, "unipeak_amd", "lib", f"libunipeak_hip_{sys.argv[2]}.so"), sys.argv[3:])
    else:
        build_all(force="--force" in sys.argv)
