#!/bin/bash
cd $GRAFT_REPO_ROOT
VR_NOLIST=1 timeout -k 10 200 python tools_dbg/cw.py && VR_WW_REFILL=64 timeout -k 10 200 python tools_dbg/cw.py
