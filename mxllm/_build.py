"""In-tree build of the mxllm native extension for gfx950 (MI355X).

No JIT cache and no hipify: every ``csrc/kernels/*.hip`` file is compiled
with ``hipcc --offload-arch=gfx950`` into an object, ``csrc/*.cpp`` (the torch
op bindings and the C++ runtime) with the host compiler, and everything is
linked into ``mxllm/_C.so`` next to this file, so the built library travels
with the repo snapshot to the GPU box.

The HIP runtime is taken from torch's own ``torch/lib/libamdhip64.so``
(same SONAME ``libamdhip64.so.7`` as /opt/rocm's), so the extension and torch
share one runtime instance in-process.

Usage: ``python -m mxllm._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shlex
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "build", "obj")
LIB_PATH = os.path.join(ROOT, "mxllm", "_C.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("MXLLM_ARCH", "gfx950")


# per-kernel-file compiler options (A/B experiments: MXLLM_FILE_FLAGS="file.hip=-opt1 -opt2;other.hip=...")
PER_FILE_HIP_FLAGS: dict[str, list[str]] = {}
for _item in filter(None, os.environ.get("MXLLM_FILE_FLAGS", "").split(";")):
    _f, _, _opts = _item.partition("=")
    PER_FILE_HIP_FLAGS.setdefault(_f.strip(), []).extend(shlex.split(_opts))


def _torch_paths():
    import torch  # noqa: F401  (only for its install location)

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash(paths, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(shlex.quote(c) for c in cmd) + "\n" + r.stdout)
    return r.stdout


def _check_loadable(path: str) -> None:
    """dlopen the fresh library in a child process (RTLD_NOW): an unresolved symbol —
    e.g. a kernel whose host launch stub the compiler dropped — fails the build here
    instead of at import on the GPU box."""
    code = f"import ctypes, os; ctypes.CDLL({path!r}, mode=os.RTLD_NOW)"
    r = subprocess.run([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        os.remove(path)
        raise RuntimeError(f"built library does not load: {r.stderr.strip()[-600:]}")


def _attn_bwd_counted_wait_ok(asm: str) -> tuple[bool, str]:
    """ISA invariant of the attention backward's counted end-of-tile wait: every
    ``s_waitcnt vmcnt(4) lgkmcnt(0)`` in front of an ``s_barrier`` must have at least 4 vector-memory
    instructions (the dS^T stores) between it and the last LDS-DMA issue before it -- then, with
    in-order retirement, vmcnt(4) implies the DMA landed.  Returns (ok, detail)."""
    import re

    found = 0
    for fn in re.findall(r"^(_ZN2mx16attn_bwd8_kernel\w+):", asm, re.M):
        i = asm.index(fn + ":")
        j = asm.index(".Lfunc_end", i)
        lines = [x.strip() for x in asm[i:j].splitlines()]
        for k, line in enumerate(lines):
            if not line.startswith("s_waitcnt vmcnt(4) lgkmcnt(0)") or k + 1 >= len(lines) or lines[k + 1] != "s_barrier":
                continue
            found += 1
            n, kk = 0, k - 1
            while kk >= 0 and not (("buffer_load" in lines[kk] and " lds" in lines[kk]) or "global_load_lds" in lines[kk]):
                if re.match(r"(global|buffer|scratch|flat)_(store|load|atomic)", lines[kk]):
                    n += 1
                kk -= 1
            if n < 4:
                return False, f"{fn}: {n} vector-memory ops between the last LDS-DMA and the counted wait"
    if found == 0:
        # the counted-wait schedule is compiled in (the check runs only on that build) but no
        # ``vmcnt(4) lgkmcnt(0)`` + barrier pair survived codegen (merged / reordered by the waitcnt
        # pass): nothing was verified, so take the safe schedule
        return False, "no counted wait found in the attn_bwd8 kernels (nothing verified)"
    return True, f"{found} counted waits checked"


# post-compile ISA checks: file -> (check(asm) -> (ok, detail), fallback compiler flag)
ISA_CHECKS = {"attn_bwd.hip": (_attn_bwd_counted_wait_ok, "-DMXLLM_ATTN_BWD_NO_COUNTED_WAIT")}


def _compile_checked(src: str, obj: str, cmd: list[str], flags: list[str]) -> str:
    """Compile; for a file with an ISA check, also emit its device assembly and verify it -- on a
    failed check recompile with the check's fallback flag (the safe, slower schedule)."""
    out = _run(cmd)
    chk = ISA_CHECKS.get(os.path.basename(src))
    if chk is None:
        return out
    fn, fallback = chk
    asm_path = obj + ".s"
    _run([os.path.join(ROCM, "bin", "hipcc")] + flags + ["-S", "--offload-device-only", src, "-o", asm_path])
    with open(asm_path) as f:
        ok, detail = fn(f.read())
    os.remove(asm_path)
    if ok:
        return out + f"\n[isa check {os.path.basename(src)}] ok: {detail}"
    print(f"[mxllm build] WARNING: ISA check of {os.path.basename(src)} failed ({detail}); "
          f"rebuilding with {fallback}", file=sys.stderr, flush=True)
    return _run([os.path.join(ROCM, "bin", "hipcc")] + flags + [fallback, "-c", src, "-o", obj])


def build(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    inc, tlib, abi = _torch_paths()
    os.makedirs(OUT_DIR, exist_ok=True)
    hdrs = sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    py_inc = sysconfig.get_paths()["include"]

    hip_flags = [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
        "-ffp-contract=fast", "-Wno-unused-result", f"-I{CSRC}", f"-I{os.path.join(CSRC, 'kernels')}",
    ]
    cxx_flags = [
        "-O3", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_C", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}", f"-I{ROCM}/include",
        f"-I{py_inc}", "-Wno-deprecated-declarations", "-Wno-unused-parameter",
    ] + [f"-I{p}" for p in inc]

    jobs_list = []
    for src in hip_srcs:
        flags = hip_flags + PER_FILE_HIP_FLAGS.get(os.path.basename(src), [])
        key = _hash([src] + hdrs, " ".join(flags))
        obj = os.path.join(OUT_DIR, os.path.basename(src) + f".{key}.o")
        cmd = [os.path.join(ROCM, "bin", "hipcc")] + flags + ["-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd, flags))
    for src in cpp_srcs:
        key = _hash([src] + hdrs, " ".join(cxx_flags))
        obj = os.path.join(OUT_DIR, os.path.basename(src) + f".{key}.o")
        cmd = ["g++"] + cxx_flags + ["-c", src, "-o", obj]
        jobs_list.append((src, obj, cmd, None))

    todo = [j for j in jobs_list if force or not os.path.exists(j[1])]
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = {ex.submit(_compile_checked if fl is not None else (lambda s_, o_, c_, f_: _run(c_)), s, o, c, fl): s
                    for (s, o, c, fl) in todo}
            for f in cf.as_completed(futs):
                out = f.result()
                if verbose:
                    print(f"[mxllm build] compiled {os.path.relpath(futs[f], ROOT)}", flush=True)
                    for line in out.splitlines():
                        if line.startswith("[isa check"):
                            print("[mxllm build] " + line[1:].replace("]", ":", 1), flush=True)
    objs = [j[1] for j in jobs_list]
    link_key = _hash([], "|".join(objs))
    stamp = LIB_PATH + ".stamp"
    if force or not os.path.exists(LIB_PATH) or not os.path.exists(stamp) or open(stamp).read() != link_key:
        tmp = LIB_PATH + ".tmp"
        cmd = (["g++", "-shared", "-o", tmp] + objs + [
            f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            f"{tlib}/libamdhip64.so", f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed",
        ])
        _run(cmd)
        _check_loadable(tmp)
        os.replace(tmp, LIB_PATH)
        with open(stamp, "w") as f:
            f.write(link_key)
        if verbose:
            print(f"[mxllm build] linked {os.path.relpath(LIB_PATH, ROOT)}", flush=True)
    _write_buildinfo(hip_srcs + cpp_srcs, hdrs, hip_flags, cxx_flags, len(todo), link_key)
    # drop stale objects from older source versions
    keep = set(objs)
    for o in glob.glob(os.path.join(OUT_DIR, "*.o")):
        if o not in keep:
            try:
                os.remove(o)
            except OSError:
                pass
    return LIB_PATH


def _write_buildinfo(srcs, hdrs, hip_flags, cxx_flags, compiled: int, link_key: str) -> None:
    """Provenance record next to the library (``mxllm/_C.buildinfo.json``): what was
    compiled, with which compiler/flags, and a hash of every source that went in."""
    import json
    import time

    try:
        ver = subprocess.run([os.path.join(ROCM, "bin", "hipcc"), "--version"], stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True).stdout.strip().splitlines()
    except OSError:
        ver = []
    info = {
        "library": os.path.relpath(LIB_PATH, ROOT),
        "arch": ARCH,
        "built_at_unix": int(time.time()),
        "objects_compiled_this_build": compiled,
        "objects_total": len(srcs),
        "link_key": link_key,
        "sources_sha1_16": _hash(srcs + hdrs, ""),
        "sources": [os.path.relpath(x, ROOT) for x in srcs],
        "hipcc": ver[:2],
        "hip_flags": hip_flags,
        "cxx_flags": [f for f in cxx_flags if not f.startswith("-I")],
    }
    with open(LIB_PATH.replace(".so", ".buildinfo.json"), "w") as f:
        json.dump(info, f, indent=1)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 8))
    a = ap.parse_args(argv)
    print(build(force=a.force, jobs=a.j, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
