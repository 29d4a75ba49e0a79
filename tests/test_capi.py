"""The C-ABI library: it loads, it exports every entry point include/ccmi.h declares, and the host-only entry
points (defaults, the RandomCluster fixture) behave. No compute call is made here (no GPU in this container)."""
import ctypes as C
import os
import re
import subprocess

import pytest
import torch

import ccmi
from oracle_binding import OracleCluster, desc_arrays

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ccmi.h")
LIB = os.path.join(REPO, "cruise-control_amd", "libccmi.so")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ccmi_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def product_lib():
    subprocess.run(["make", "-C", os.path.join(REPO, "cruise-control_amd"), "-j8"], check=True, capture_output=True)
    return ccmi.Library.get(LIB)


def test_header_declares_binding_symbols():
    assert _declared() == sorted(ccmi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(product_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing
    for s in _declared():
        assert getattr(product_lib.lib, s) is not None


def test_library_is_gfx950_code_object(product_lib):
    """The product library embeds an amdgcn code object built for gfx950."""
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_abi_version_and_defaults(product_lib):
    L = product_lib.lib
    assert L.ccmi_abi_version() >= 1
    c = ccmi.ConstraintStruct()
    L.ccmi_default_constraint(C.byref(c))
    assert list(c.capacity_threshold) == [0.7, 0.8, 0.8, 0.8]
    assert list(c.resource_balance_percentage) == [1.1] * 4
    assert c.replica_balance_percentage == 1.1
    p = ccmi.RandomClusterProps()
    L.ccmi_default_random_cluster_props(C.byref(p))
    assert (p.num_racks, p.num_brokers, p.num_replicas, p.num_topics) == (10, 40, 50001, 3000)


@pytest.mark.parametrize("props", [dict(num_racks=5, num_brokers=20, num_replicas=6000, num_topics=300),
                                   dict(num_racks=3, num_brokers=10, num_replicas=3000, num_topics=100,
                                        num_dead_brokers=2),
                                   dict(num_racks=3, num_brokers=10, num_replicas=3000, num_topics=100,
                                        num_dead_brokers=2, rack_aware=1),
                                   dict()])
def test_random_cluster_fixture_matches_oracle(product_lib, oracle_lib, props):
    """The product's RandomCluster (host code) emits the same flattened cluster the oracle generator builds."""
    buf = ccmi.RandomCluster.generate(product_lib, **props)
    assert desc_arrays(buf.desc) == OracleCluster.random(**props).export()


def test_random_cluster_bad_input(product_lib):
    with pytest.raises(ccmi.IllegalArgumentException):
        ccmi.RandomCluster.generate(product_lib, num_replicas=10, min_replication=3, max_replication=3)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device failure mode")
def test_session_fails_loudly_without_gfx950(product_lib):
    buf = ccmi.RandomCluster.generate(product_lib, num_brokers=6, num_racks=3, num_replicas=300, num_topics=10)
    with pytest.raises(ccmi.DeviceError):
        ccmi.ClusterModel.from_buffers(buf, device=0)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ccmi.DeviceError):
        ccmi.Library(str(tmp_path / "libccmi.so"))
