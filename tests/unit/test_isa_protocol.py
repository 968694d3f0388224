"""The cross-device memory-model sequence of the xGMI data plane, as built.

The fused all-reduce jobs (csrc/kernels/comm_jobs.h: ``comm_publish`` /
``comm_wait``) and the standalone push kernel (p2p_allreduce.hip) rely on
system-scope cache-control bits and waits that only the compiler's output
shows. This CPU test reads them out of the built ``_C.so`` (unbundled with
llvm-objcopy, disassembled with llvm-objdump; nothing from the file runs), so
a flag or compiler change that weakens them fails here instead of on the
first 8-GPU run. The sequences are documented in docs/KERNELS.md
("Cross-device memory-model sequence").

Reference counterpart: the per-step all-reduce these kernels replace
(/root/reference/vae-hpo.py:72, DDP -> NCCL).
"""
import os

import pytest

from multidisttorch_amd.obs import isa

pytestmark = pytest.mark.skipif(not (isa.tools_available() and os.path.exists(isa.SO)),
                                reason="needs the built _C.so and the ROCm llvm tools")


@pytest.fixture(scope="module")
def sites():
    out = {}
    for name, sub in isa.COMM_KERNELS.items():
        text = isa.disassemble(sub)
        assert text is not None, f"{name} not found in the gfx950 code objects of {isa.SO}"
        out[name] = isa.protocol_sites(text)
    return out


def test_code_objects_are_gfx950():
    cos = isa.gfx950_code_objects()
    assert cos and all(c[:4] == b"\x7fELF" for c in cos)


@pytest.mark.parametrize("kernel", sorted(isa.COMM_KERNELS))
def test_publish_drains_data_stores_before_any_flag(sites, kernel):
    # release fence at system scope, then vmcnt(0) (every data store of the
    # wave acknowledged), then the workgroup barrier: no lane writes a flag
    # before every wave's stores into the peer's region have completed
    s = sites[kernel]["publish_drain"]
    assert s, sites[kernel]
    for site in s:
        assert site[0] == "buffer_wbl2 sc0 sc1" and site[-1] == "s_barrier"


@pytest.mark.parametrize("kernel", sorted(isa.COMM_KERNELS))
def test_flag_is_a_system_scope_release_store(sites, kernel):
    s = sites[kernel]["flag_release"]
    assert s, sites[kernel]
    for wb, st in s:
        assert wb == "buffer_wbl2 sc0 sc1" and "store_dword" in st and st.endswith("sc0 sc1")


@pytest.mark.parametrize("kernel", sorted(isa.COMM_KERNELS))
def test_poll_is_a_system_scope_acquire_load(sites, kernel):
    s = sites[kernel]["poll_acquire"]
    assert s, sites[kernel]
    for ld, wait, inv in s:
        assert "load_dword" in ld and ld.endswith("sc0 sc1") and "vmcnt(0)" in wait and inv == "buffer_inv sc0 sc1"


@pytest.mark.parametrize("kernel", sorted(isa.COMM_KERNELS))
def test_acquire_fence_after_the_poll(sites, kernel):
    s = sites[kernel]["fence_acquire"]
    assert s, sites[kernel]


def test_every_publish_has_its_wait(sites):
    # comm_jobs.h: one publish + one wait per form (one-shot flag 2e-1, two-shot
    # all-gather flag 2e): each publish site pairs with a poll and a fence site
    j = sites["jobs_multi_k"]
    assert len(j["publish_drain"]) == len(j["flag_release"]) == len(j["poll_acquire"]) == len(j["fence_acquire"]) >= 2


@pytest.fixture(scope="module")
def dep():
    text = isa.disassemble(isa.DEP_KERNEL)
    assert text is not None, f"{isa.DEP_KERNEL} not found in {isa.SO}"
    return isa.dep_sites(text)


def test_dependent_jobs_poll_and_count_with_global_agent_accesses(dep):
    # conv_jobs.hip dep_wait / dep_signal: the bounded poll is a relaxed agent
    # (sc1) GLOBAL load beside its s_sleep; the producer's counter add follows
    # its drain (vmcnt(0) + barrier) and, for plain-store producers, an agent
    # release; no flat access carries the agent bit
    assert dep["poll"], dep
    assert dep["drain_add"], dep
    assert dep["release_add"], dep
    assert not dep["flat_agent"], dep["flat_agent"]


def test_dependent_finalize_reads_slabs_past_l1(dep):
    # FinalizeArgs.dep: the slabs handed off inside the launch are read with
    # sc1 buffer loads (16-B vec4 units and 4-B scalar units)
    assert any("dwordx4" in o for o in dep["sc1_loads"]), dep["sc1_loads"]
    assert any("dwordx4" not in o for o in dep["sc1_loads"]), dep["sc1_loads"]
