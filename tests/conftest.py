"""pytest configuration: the `gpu` marker and import paths.

CPU tests (-m "not gpu") check the oracle against the reference's golden
vectors, the host logic, and that libmapf.so loads and exports every symbol
include/mapf.h declares.  GPU tests (-m gpu) are the parity tests proper.
"""
import os
import sys

# before anything initialises the HIP runtime: captured memsets replay once under packet capture
# (primal-ppo_amd/mapf_amd/__init__.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "primal-ppo_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
