#!/usr/bin/env python3
"""Oracle (oracle/refchol.c restatement of the reference chol(), per-row workspace kept)
timed in this container on the SURVEY.md section 6 inputs, median of N runs, 1 core.
The reference itself is unbuildable here, so the ratio is taken
against the survey's measured reference times (same container family, 1 core)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import sparsecholesky_amd as sc  # noqa: E402

SURVEY_MS = {"bcsstk01": 0.04, "1138_bus": 2.70, "lap16_nd": 55.1, "lap24_nd": 681.0, "lap32_nd": 4700.0,
             "lap48_nd": 68800.0}


def main():
    cases = [("bcsstk01", 9), ("1138_bus", 9), ("lap16_nd", 9), ("lap24_nd", 3), ("lap32_nd", 3)]
    if "--with-48" in sys.argv:
        cases.append(("lap48_nd", 1))
    for name, reps in cases:
        if name.startswith("lap"):
            A = sc.laplacian3d(int(name[3:5]))
        else:
            A = sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests", "golden", name + ".mtx"))
        # whole chol() call (symbolic + numeric, as the reference's chol() does), timed in C
        ts = []
        for _ in range(reps):
            st, sec = oracle.time_chol(A, reps=1, faithful_workspace=True)
            assert st == 0
            ts.append(sec * 1e3)
        med = statistics.median(ts)
        print(json.dumps({"matrix": name, "oracle_ms_median": round(med, 4), "runs": reps,
                          "reference_ms_survey": SURVEY_MS[name],
                          "oracle_over_reference": round(med / SURVEY_MS[name], 3)}), flush=True)


if __name__ == "__main__":
    main()
