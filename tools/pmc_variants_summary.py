#!/usr/bin/env python3
"""Summarise tools/pmc_variants.sh output: cycles, clock, MFMA busy, VALU/LDS instructions per
tile (9537 tiles per SIMD on C3) of each k_moments_ws variant.  Usage: <tag> <variant>..."""
import csv, json, sys, os
tag=sys.argv[1]
for v in sys.argv[2:]:
    agg={}
    with open(f"gpurun_out/pmcv_{tag}/{v}/pmc_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if "k_moments" in r["Kernel_Name"]:
                agg[r["Counter_Name"]]=agg.get(r["Counter_Name"],0)+float(r["Counter_Value"])
    j=json.load(open(f"gpurun_out/pmcv_{tag}/{v}.json")); ms=j["kernels_ms"]["moments"]
    g=agg["GRBM_GUI_ACTIVE"]/8; tiles=9537*1024
    print(f"{v:12s} ms {ms:7.2f} Mcyc {g/1e6:6.1f} GHz {g/ms/1e6:5.3f} mfma% {agg['SQ_VALU_MFMA_BUSY_CYCLES']/1024/g*100:5.1f} valu/tile {agg['SQ_INSTS_VALU']/tiles:6.1f} lds/tile {agg['SQ_INSTS_LDS']/tiles:6.1f} ovh cyc/tile {(g-agg['SQ_VALU_MFMA_BUSY_CYCLES']/1024)/9537:7.1f}")
