#!/usr/bin/env python3
"""Compact kbench JSON lines from stdin: chain (truncated), shape, ms."""
import json
import sys

for line in sys.stdin:
    if line.startswith("{"):
        r = json.loads(line)
        print(f"{r['chain'][:24]:24s} {r['shape']:14s} {r['ms']:.4f} ms")
