import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dalle2-video_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP path)")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def parity_log(request):
    """record(**values): prints the observed errors and, when DV_PARITY_LOG
    names a file, appends them as one JSON line (test id + values) so the
    worst observed error of every tolerance-checked comparison is kept."""
    path = os.environ.get("DV_PARITY_LOG")

    def record(**values):
        line = {"test": request.node.nodeid, **values}
        print(json.dumps(line))
        if path:
            with open(path, "a") as f:
                f.write(json.dumps(line) + "\n")
    return record
