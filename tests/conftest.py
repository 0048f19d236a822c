"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on any host (oracle vs golden vectors, host logic, C-ABI
load/exports, gloo multi-process); `-m gpu` runs the parity tests proper on an
MI355X through the C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "network-stack_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


def pytest_sessionstart(session):
    # Bring the checker (oracle) and the product library up to date in-tree before any test loads them. make is
    # incremental: a no-op when the built files match their sources, so a stale pushed .so never runs and an
    # up-to-date one is not rebuilt.
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "network-stack_amd")])
