import datetime
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Parity audit records (VERDICT r1 "make parity auditable"): GPU parity tests append one dict per
# case — rows compared, rows that differ from the reference, rows the certificate flags — and the
# session writes them to $GR_PARITY_OUT (default gpurun_out/parity_counts.json, which gpurun copies
# back; the committed copy lives under profiles/).
_PARITY = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU")
    return torch.device("cuda:0")


@pytest.fixture
def parity_log(request):
    """``parity_log(**fields)`` records one parity count (JSON-serialisable values) for the audit
    file, tagged with the test id."""
    def rec(**kw):
        row = {"test": request.node.nodeid}
        for k, v in kw.items():
            row[k] = v.item() if hasattr(v, "item") and getattr(v, "ndim", 0) == 0 else v
        _PARITY.append(row)
        print("\nPARITY " + json.dumps(row, default=float))
    return rec


def pytest_sessionfinish(session, exitstatus):
    if not _PARITY:
        return
    path = os.environ.get("GR_PARITY_OUT", os.path.join(ROOT, "gpurun_out", "parity_counts.json"))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    info = {"written": datetime.datetime.utcnow().isoformat() + "Z", "exitstatus": int(exitstatus)}
    try:
        import torch
        info["torch"] = torch.__version__
        if torch.cuda.is_available():
            info["device"] = torch.cuda.get_device_name(0)
    except Exception:  # pragma: no cover - the audit file must not fail the session
        pass
    with open(path, "w") as f:
        json.dump({"info": info, "records": _PARITY}, f, indent=1, default=float)
