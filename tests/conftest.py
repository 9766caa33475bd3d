import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kubernetes-rca-system_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# (Rounds 5 ran the GPU tests with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0: with the runtime's graph packet
# capture on, a captured solve replayed wrong after ~300 later eager launches.  The cause was the
# solve's hipMemsetAsync nodes, whose replays read stale staging bytes (tools/graph_replay_probe.py,
# R6a); the solve zeroes with kernels now, and the tests run with the runtime's default setting.)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libkrca.so on the device)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_report_header(config):
    """The libkrca build the run loads (path, krca_version(), SHA-256 prefix), in the run's header."""
    try:
        from krca import native
        return f"libkrca: {native.library_info()}"
    except Exception as e:  # noqa: BLE001  (no build yet: the CPU suite reports it)
        return f"libkrca: not loaded ({e})"
