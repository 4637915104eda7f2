#!/usr/bin/env python3
"""Exhaustive check of the kernels' reciprocal (rt_device.h rcp_nr) on the GPU: prints the
mismatch count per biased exponent against the correctly rounded 1.0f / x (all floats)."""
import importlib.util
import json
import os
import sys

import torch  # noqa: F401  (first: share torch's HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("rtm", os.path.join(ROOT, "cpp-11-ray-trace-march-framework_amd", "__init__.py"))
rtm = importlib.util.module_from_spec(spec)
sys.modules["rtm"] = rtm
spec.loader.exec_module(rtm)
bad = rtm.debug_rcp_check(0)
print(json.dumps({"total_bad": int(bad.sum()), "bad_by_exponent": {int(e): int(c) for e, c in enumerate(bad) if c}}))
