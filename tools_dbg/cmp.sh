#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools_dbg/cmp.py /tmp/ww.npy && VR_SECONDARY=s timeout -k 10 200 python tools_dbg/cmp.py /tmp/s.npy && python tools_dbg/cmp.py cmp /tmp/ww.npy /tmp/s.npy
