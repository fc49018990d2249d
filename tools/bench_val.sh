#!/bin/bash
# print "<label> <images|sequences per s> <ms/step>" from a bench.py log (last JSON line)
tail -1 "$2" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["value"], d["ms_per_step"])' "$1"
