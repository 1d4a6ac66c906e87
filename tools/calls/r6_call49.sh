#!/bin/bash
# round 6, call 49: DWA step at 256 agents, 1 / 2 / 4 workgroups per agent (k-split kernel)
# result: 256 agents, parts 1 / 2 / 4: 195.6 / 222.0 / 222.8 us per step (wrapper span) -- one workgroup per agent stays
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 300 python3 -u tools/dwa_split_probe.py
