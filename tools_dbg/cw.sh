#!/bin/bash
cd $GRAFT_REPO_ROOT
VR_WW_PROF=1 VR_WW_COUNT=1 timeout -k 10 200 python tools_dbg/cw.py && VR_WW_PROF=2 VR_WW_COUNT=1 timeout -k 10 200 python tools_dbg/cw.py
