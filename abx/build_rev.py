#!/usr/bin/env python3
"""Build build_ab/NAME.so from a git revision's mp3_amd/csrc (A/B against HEAD or
any commit).  Usage: python abx/build_rev.py NAME REV"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mp3_amd import _build  # noqa: E402

name, rev = sys.argv[1], sys.argv[2]
root = tempfile.mkdtemp(prefix="rev_")
tar = subprocess.run(["git", "archive", rev, "mp3_amd/csrc", "include"], check=True, capture_output=True).stdout
subprocess.run(["tar", "-x", "-C", root], input=tar, check=True)
_build.compile_hip(os.path.join(root, "mp3_amd", "csrc"), "build_ab/%s.so" % name, os.path.join(root, "obj"))
print("build_ab/%s.so from %s" % (name, rev))
