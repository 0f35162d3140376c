"""pytest configuration: `gpu` marks tests that need an MI355X (run with -m gpu)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _oracle_single_thread():
    # the oracle's emulated ranks run as OpenMP threads; the test problems are tiny
    try:
        from oracle import oracle

        oracle.set_threads(1)
    except Exception:
        pass


_oracle_single_thread()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: large-grid property test")
