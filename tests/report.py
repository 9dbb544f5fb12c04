"""Parity statistics the GPU tests print (silhouette flip counts, PSNR, max errors).

Each call prints one JSON line (visible with ``pytest -s`` or in the failure output) and, when
``NRT_REPORT`` names a file, appends the line to it, so a GPU run can keep the numbers
(``NRT_REPORT=gpurun_out/parity_report.jsonl``)."""
import json
import os


def report(test, **values):
    line = json.dumps({"test": test, **{k: _plain(v) for k, v in values.items()}})
    print("PARITY " + line, flush=True)
    path = os.environ.get("NRT_REPORT")
    if path:
        with open(path, "a") as fh:
            fh.write(line + "\n")
    return values


def _plain(v):
    if hasattr(v, "item"):
        return v.item()
    return v
