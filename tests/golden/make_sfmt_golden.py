#!/usr/bin/env python3
"""Extracts the SFMT19937 known-answer vector of the reference's own test
(src/tests/test_random.cpp:433-508, TestRandom::test00_validate: the first
outputs of Random(4321)::nextULong) into sfmt19937_kat.json.  Data only; run
in the builder container where /root/reference exists."""
import json
import os
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else '/root/reference/src/tests/test_random.cpp'
text = open(src).read()
body = text[text.index('void TestRandom::test00_validate()'):]
body = body[:body.index('};')]
vals = [int(v, 16) for v in re.findall(r'0x([0-9a-fA-F]{16})ULL', body)]
seed = int(re.search(r'new Random\((\d+)\)', text[text.index('void TestRandom::test00_validate()'):]).group(1))
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'sfmt19937_kat.json')
json.dump({'source': 'src/tests/test_random.cpp:433-508 (test00_validate)', 'seed': seed,
           'next_ulong': ['0x%016x' % v for v in vals]}, open(out, 'w'), indent=0)
print('%d values, seed %d -> %s' % (len(vals), seed, out))
