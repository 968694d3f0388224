"""ISA-level records of the built gfx950 code objects (CPU only).

The fused xGMI all-reduce jobs (csrc/kernels/comm_jobs.h) and the standalone
push kernel (csrc/kernels/p2p_allreduce.hip) hand data between GPUs with a
release/acquire protocol at SYSTEM scope: data stores into the peer's
uncached region, ``s_waitcnt vmcnt(0)``, a workgroup barrier, then a
system-scope release store of the flag; the consumer polls the flag with
system-scope acquire loads. Whether that protocol holds across devices is
decided by the cache-control bits and waits the compiler actually emitted,
so this module reads them out of ``multidisttorch_amd/_C.so`` itself:

* ``gfx950_code_objects`` unbundles the ``.hip_fatbin`` section (clang
  offload bundles, one per HIP translation unit) without running anything
  from the file;
* ``disassemble`` runs ``llvm-objdump`` on the code object that defines a
  kernel;
* ``protocol_sites`` finds the publish / poll / acquire sequences
  (docs/KERNELS.md "Cross-device memory-model sequence") so a test can assert
  they are still there after a flag or compiler change.

Reference counterpart: the per-step all-reduce these jobs replace,
``loss.backward()`` -> DDP -> NCCL (/root/reference/vae-hpo.py:72), whose
ordering lives inside RCCL.

Run ``python -m multidisttorch_amd.obs.isa`` to print the sequences.
"""

from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile
from typing import Dict, List, Optional

LLVM_BIN = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")
SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# kernels whose cross-device protocol is recorded (mangled-name substrings)
COMM_KERNELS = {"jobs_multi_k": "jobs_multi_k", "p2p_allreduce_k": "p2p_allreduce_k"}


def tools_available() -> bool:
    return all(os.path.exists(os.path.join(LLVM_BIN, t)) for t in ("llvm-objcopy", "llvm-objdump", "llvm-readelf"))


def gfx950_code_objects(so_path: str = SO, arch: str = "gfx950") -> List[bytes]:
    """The ``arch`` device code objects bundled into ``so_path``."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(LLVM_BIN, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", so_path,
                        os.path.join(td, "copy.o")], check=True, capture_output=True)
        with open(fat, "rb") as f:
            d = f.read()
    out = []
    for p in range(0, len(d) - len(_MAGIC), 8):
        if d[p:p + len(_MAGIC)] != _MAGIC:
            continue
        n = struct.unpack_from("<Q", d, p + 24)[0]
        q = p + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", d, q)
            q += 24
            triple = d[q:q + tl].decode(errors="replace")
            q += tl
            if triple.endswith(arch) or f"--{arch}" in triple:
                out.append(d[p + off:p + off + size])
    return out


def disassemble(kernel: str, so_path: str = SO) -> Optional[str]:
    """``llvm-objdump -d`` of the kernel whose mangled name contains ``kernel``."""
    for co in gfx950_code_objects(so_path):
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "co.elf")
            with open(path, "wb") as f:
                f.write(co)
            syms = subprocess.run([os.path.join(LLVM_BIN, "llvm-readelf"), "-s", "--wide", path],
                                  capture_output=True, text=True).stdout
            names = sorted({l.split()[-1] for l in syms.splitlines() if " FUNC " in l and kernel in l.split()[-1]})
            if not names:
                continue
            return subprocess.run([os.path.join(LLVM_BIN, "llvm-objdump"), "-d",
                                   f"--disassemble-symbols={names[0]}", path],
                                  capture_output=True, text=True, check=True).stdout
    return None


def _ops(text: str) -> List[str]:
    """Instruction lines without the address/encoding comment."""
    ops = []
    for l in text.splitlines():
        l = l.strip()
        if not l or l.endswith(":") or l.startswith(("Disassembly", ";")) or "file format" in l:
            continue
        ops.append(l.split("//")[0].strip())
    return [o for o in ops if o]


_SYS = r"\bsc0 sc1\b"
_WB = re.compile(r"^buffer_wbl2 sc0 sc1$")
_INV = re.compile(r"^buffer_inv sc0 sc1$")
_STORE = re.compile(r"^(flat|global)_store_dword\b.*" + _SYS)
_LOAD = re.compile(r"^(flat|global)_load_dword\b.*" + _SYS)
_WAIT_VM0 = re.compile(r"^s_waitcnt\b.*vmcnt\(0\)")


def protocol_sites(text: str, window: int = 4) -> Dict[str, list]:
    """Instruction windows of the cross-device protocol in a disassembly:

    * ``publish_drain``: ``buffer_wbl2 sc0 sc1`` (release fence, system scope)
      followed by ``s_waitcnt vmcnt(0)`` and ``s_barrier`` -- every wave's
      data stores have completed before any flag is written;
    * ``flag_release``: ``buffer_wbl2 sc0 sc1`` directly followed by a
      ``*_store_dword ... sc0 sc1`` (the flag: system-scope release store);
    * ``poll_acquire``: ``*_load_dword ... sc0 sc1`` then ``s_waitcnt
      vmcnt(0)`` then ``buffer_inv sc0 sc1`` (system-scope acquire load);
    * ``fence_acquire``: ``s_barrier``, ``s_waitcnt vmcnt(0)``, ``buffer_inv
      sc0 sc1`` (the acquire fence after the poll, before reading peer data).
    """
    ops = _ops(text)
    sites: Dict[str, list] = {"publish_drain": [], "flag_release": [], "poll_acquire": [], "fence_acquire": []}
    for i, o in enumerate(ops):
        nxt = ops[i + 1:i + 1 + window]
        if _WB.match(o):
            if nxt and _STORE.match(nxt[0]):
                sites["flag_release"].append([o, nxt[0]])
            w = [j for j, x in enumerate(nxt) if _WAIT_VM0.match(x)]
            b = [j for j, x in enumerate(nxt) if x == "s_barrier"]
            if w and b and w[0] < b[0]:
                sites["publish_drain"].append([o] + nxt[:b[0] + 1])
        if _LOAD.match(o) and len(nxt) >= 2 and _WAIT_VM0.match(nxt[0]) and _INV.match(nxt[1]):
            sites["poll_acquire"].append([o] + nxt[:2])
        if o == "s_barrier" and len(nxt) >= 2 and _WAIT_VM0.match(nxt[0]) and _INV.match(nxt[1]):
            sites["fence_acquire"].append([o] + nxt[:2])
    return sites


# the in-launch dependency protocol of the dependent multi-job kernel
# (conv_jobs.hip dep_wait / dep_signal, FinalizeArgs.dep, batch_gather_dep_body)
DEP_KERNEL = "jobs_multi_kILb1E"
_AGENT_LD = re.compile(r"^global_load_dword\S*\b.*\bsc1$")
_AGENT_ADD = re.compile(r"^global_atomic_add\b")
_SC1_BUF_LD = re.compile(r"^buffer_load_dword(x4)?\b.*\bsc1$")
_FLAT_AGENT = re.compile(r"^flat_(load|store|atomic)\S*\b(?!.*\bsc0\b).*\bsc1\b")


def dep_sites(text: str, window: int = 40) -> Dict[str, list]:
    """Instruction windows of the dependent launch's hand-off protocol:

    * ``poll``: an agent-scope ``global_load_dword ... sc1`` within a few
      instructions of an ``s_sleep`` (the bounded counter poll);
    * ``release_add``: ``buffer_wbl2 sc1`` (agent release, plain-store
      producers), ``s_waitcnt vmcnt(0)``, then a ``global_atomic_add`` (the
      counter add) inside ``window`` instructions;
    * ``drain_add``: ``s_waitcnt vmcnt(0)`` (explicit drain), ``s_barrier``
      within 3 instructions, then a ``global_atomic_add`` inside ``window``;
    * ``sc1_loads``: ``buffer_load_dword[x4] ... sc1`` (slab reads past L1);
    * ``flat_agent``: flat accesses with agent-scope ``sc1`` (must be none:
      every hand-off access is global or buffer).
    """
    ops = _ops(text)
    out: Dict[str, list] = {"poll": [], "release_add": [], "drain_add": [], "sc1_loads": [], "flat_agent": []}
    for i, o in enumerate(ops):
        nxt = ops[i + 1:i + 1 + window]
        if _AGENT_LD.match(o) and any(x.startswith("s_sleep") for x in ops[max(0, i - 3):i + 4]):
            out["poll"].append(o)
        if o == "buffer_wbl2 sc1" and nxt and _WAIT_VM0.match(nxt[0]):
            a = [x for x in nxt if _AGENT_ADD.match(x)]
            if a:
                out["release_add"].append([o, nxt[0], a[0]])
        if _WAIT_VM0.match(o) and "s_barrier" in nxt[:3]:
            a = [x for x in nxt if _AGENT_ADD.match(x)]
            if a:
                out["drain_add"].append([o, "s_barrier", a[0]])
        if _SC1_BUF_LD.match(o):
            out["sc1_loads"].append(o)
        if _FLAT_AGENT.match(o):
            out["flat_agent"].append(o)
    return out


def main():
    for name, sub in COMM_KERNELS.items():
        text = disassemble(sub)
        print(f"== {name}: {'not found' if text is None else str(len(_ops(text))) + ' instructions'}")
        if text is None:
            continue
        for k, v in protocol_sites(text).items():
            print(f"  {k}: {len(v)} site(s)")
            for site in v[:2]:
                print("    " + " ; ".join(site))
    text = disassemble(DEP_KERNEL)
    print(f"== {DEP_KERNEL}: {'not found' if text is None else str(len(_ops(text))) + ' instructions'}")
    if text is not None:
        for k, v in dep_sites(text).items():
            print(f"  {k}: {len(v)} site(s)")
            for site in v[:2]:
                print("    " + (" ; ".join(site) if isinstance(site, list) else site))


if __name__ == "__main__":
    main()
