#!/usr/bin/env python3
"""Alternating A/B of library builds on one box: runs tools/ntt_rate.py with MFHE_LIB = each library in turn,
`rounds` times.  usage: tools/lib_ab.py rounds lib1,lib2,... -- ntt_rate args"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
rounds = int(sys.argv[1])
libs = sys.argv[2].split(",")
args = sys.argv[sys.argv.index("--") + 1:]
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, MFHE_LIB=str(ROOT / "matrix-fhe-gpu_amd" / lib))
        p = subprocess.run([sys.executable, str(ROOT / "tools" / "ntt_rate.py"), *args], env=env, capture_output=True,
                           text=True, timeout=300)
        print(p.stdout.strip() or p.stderr[-500:], flush=True)
        if p.returncode:
            sys.exit(p.returncode)
