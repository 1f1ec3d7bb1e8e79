#!/usr/bin/env python3
"""Repeated bcsstk01 factorizations (for a kernel trace of the tiny launch): 200 eager
factorizations through one handle.  Usage: tiny_probe.py [package dir]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else ROOT)
import sparsecholesky_amd as sc  # noqa: E402

A = sc.load_matrix_market_to_csc(os.path.join(ROOT, "tests/golden/bcsstk01.mtx"))
num = sc.Numeric(sc.Symbolic(A, use_graph=0))
for _ in range(200):
    assert num.factor(A.x) == 0
print("tiny probe ok", sc.__file__)
