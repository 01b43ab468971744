"""SPEED submission export (REV/utils/submission.py, used by REV/gen_submission_multi.py):
collected poses, sorted by filename (synthetic test images first, then real), written as CSV
rows `filename, q0, q1, q2, q3, x, y, z`.  Host-side formatting, no device work."""
from __future__ import annotations

import csv
import os
from datetime import datetime


class SubmissionWriter:
    def __init__(self):
        self.test_results = []
        self.real_test_results = []

    def _append(self, filename, q, r, real):
        (self.real_test_results if real else self.test_results).append(
            {"filename": filename, "q": list(q), "r": list(r)})

    def append_test(self, filename, q, r):
        self._append(filename, q, r, real=False)

    def append_real_test(self, filename, q, r):
        self._append(filename, q, r, real=True)

    def export(self, out_dir="", suffix=None):
        sorted_test = sorted(self.test_results, key=lambda k: k["filename"])
        sorted_real = sorted(self.real_test_results, key=lambda k: k["filename"])
        suffix = datetime.now().strftime("%Y%m%d-%H%M") if suffix is None else suffix
        path = os.path.join(out_dir, f"submission_{suffix}.csv")
        with open(path, "w") as f:
            w = csv.writer(f, lineterminator="\n")
            for r in sorted_test + sorted_real:
                w.writerow([r["filename"], *(r["q"] + r["r"])])
        return path
