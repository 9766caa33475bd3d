#!/usr/bin/env python3
"""Run one pytest-style test function N times in this process (an intermittent mismatch, not a
fault: a bounded loop in one process), optionally under a libkrca knob; reports pass / fail counts
and the first failure messages.

  python tools/repeat_test.py tests/test_gpu_stream.py test_stream_window_log_overlap_and_error_path 10 [KNOB=V ...]
"""
import importlib.util
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "kubernetes-rca-system_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    path, name, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    knobs = dict(kv.split("=") for kv in sys.argv[4:])
    from krca import native
    eng = native.NativeEngine()
    for k, v in knobs.items():
        assert eng.lib.krca_tune_set(k.encode(), int(v)) == 0, k
    spec = importlib.util.spec_from_file_location("t", os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    fn = getattr(mod, name)
    ok, bad = 0, []
    for i in range(n):
        try:
            fn(eng)
            ok += 1
        except AssertionError as e:  # a mismatch: record it and go on
            bad.append((i, "".join(traceback.format_exception_only(type(e), e)).strip()[:300]))
        print(f"run {i}: {'ok' if len(bad) == 0 or bad[-1][0] != i else 'FAIL ' + bad[-1][1]}", flush=True)
    print(f"{name} {knobs}: {ok} passed, {len(bad)} failed", flush=True)


if __name__ == "__main__":
    main()
