"""Shared fixtures.

* ``dg``     — the product package (delta-compression_amd/), loaded by path
               because the directory name is not a Python identifier.
* ``orc``    — the oracle (oracle/, TEST INFRASTRUCTURE: the checker only).
* ``ref``    — the reference's own src/c compiled by oracle/Makefile, when
               present (it is built in the dev container and travels to the
               GPU box as oracle/_ref/libdelta_ref.so).

GPU tests are marked ``@pytest.mark.gpu`` and run only on an MI355X box.
"""
from __future__ import annotations

import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "delta-compression_amd")
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_product():
    if "delta_compression_amd" in sys.modules:
        return sys.modules["delta_compression_amd"]
    spec = importlib.util.spec_from_file_location(
        "delta_compression_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["delta_compression_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def dg():
    return load_product()


@pytest.fixture(scope="session")
def orc():
    import oracle as O
    return O.Oracle()


@pytest.fixture(scope="session")
def ref():
    import oracle as O
    if not O.reference_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    return O.Reference()


@pytest.fixture(scope="session")
def ctx(dg):
    return dg.Context(0)


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="session", params=["members", "chain", "auto"])
def ctx_mode(dg, request):
    """A context per onepass chain mode (DG_LIMIT_ONEPASS_MEMBERS): verified
    diagonal members first, the plain per-pair chain, or the automatic choice
    (members for large pairs; pairs whose chunks verify fewer than 2 members
    each on average, i.e. whose matches leave diagonal 0, routed to the plain
    per-pair chain after the member chain, dg_onepass.hip)."""
    c = dg.Context(0)
    c.set_limit(dg.LIMIT_ONEPASS_MEMBERS, {"members": dg.MEMBERS_ON, "chain": dg.MEMBERS_OFF,
                                           "auto": dg.MEMBERS_AUTO}[request.param])
    return c
