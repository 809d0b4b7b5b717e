#!/usr/bin/env python
"""A/B of FrozenResNetPlan.STEM_CHUNK at the headline batch: python scripts/stem_chunk_ab.py CHUNK"""
import os, sys, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import bench
from ncnet_amd.models import backbones
backbones.STEM_CHUNK = int(sys.argv[1])
bench.main(["--batch", "256", "--steps", "8", "--warmup", "3", "--inloc", "0"])
