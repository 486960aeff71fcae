import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")


def pytest_sessionstart(session):
    # Initialise torch's HIP context before any test creates a libflinkwin handle: a process whose
    # first HIP call came from the library (hipMalloc in fw_create) can see torch.cuda.is_available()
    # return False afterwards, which would skip the torch-based GPU tests of the same session.
    try:
        import torch
        torch.cuda.is_available()
    except Exception:
        pass
