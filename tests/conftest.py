import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


def pytest_collection_modifyitems(config, items):
    """GPU runs: torch (whose wheel bundles its own HIP runtime) initialises the device before
    libymerge.so's runtime does.  In the other order torch's first CUDA call in the process reports "No HIP
    GPUs are available" (seen on the box when a -k selection reached a torch-using test only after
    library-only tests); the full suite happened to initialise torch first."""
    if any(item.get_closest_marker("gpu") for item in items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass
