#!/usr/bin/env python3
"""Colour counts of the seeded-priority JP and speculative modes against the reference path (oracle only; CPU).
Writes profiles/priority_colour_counts.json.  Run from the repo root: python tools/colour_report.py"""
import sys, random, json
sys.path.insert(0,'.'); sys.path.insert(0,'tests'); sys.path.insert(0,'distributed-graph-coloring-with-pyspark_amd')
import numpy as np
from oracle import oracle
from test_oracle_omp import rmat_csr
from gcolor_amd.generators import reference_csr
def mesh(nx,ny,nz):
    idx=lambda x,y,z: x+nx*(y+ny*z)
    rp=[0]; col=[]
    for z in range(nz):
        for y in range(ny):
            for x in range(nx):
                for (dx,dy,dz) in [(-1,0,0),(1,0,0),(0,-1,0),(0,1,0),(0,0,-1),(0,0,1)]:
                    X,Y,Z=x+dx,y+dy,z+dz
                    if 0<=X<nx and 0<=Y<ny and 0<=Z<nz: col.append(idx(X,Y,Z))
                rp.append(len(col))
    return np.array(rp,np.int64), np.array(col,np.int32)
graphs=[]
for s in (0,1,2,3):
    graphs.append((f"Graph(10000,8) seed {s}",)+reference_csr(10000,8,random.Random(s)))
for sc in (12,14,16):
    graphs.append((f"R-MAT {sc} (numpy, seed {sc})",)+rmat_csr(sc,16,sc))
graphs.append(("mesh 16^3",)+mesh(16,16,16)); graphs.append(("mesh 32^3",)+mesh(32,32,32))
rows=[]
for name,rp,col in graphs:
    a=oracle.c_color(rp,col,'A')
    r={"graph":name,"ref_A":int(a['max_color'])+1,"ref_rounds":int(a['rounds'])}
    for seed in (1,2,3):
        b=oracle.c_color_prio(rp,col,priority=1,seed=seed)
        c=oracle.c_color_prio(rp,col,priority=1,seed=seed,speculative=True)
        r.setdefault("seededJP",[]).append(int(b['max_color'])+1); r.setdefault("seededJP_rounds",[]).append(int(b['rounds']))
        r.setdefault("spec",[]).append(int(c['max_color'])+1); r.setdefault("spec_rounds",[]).append(int(c['rounds']))
    d=oracle.c_color_prio(rp,col,priority=0,speculative=True)
    r["spec_ref"]=int(d['max_color'])+1; r["spec_ref_rounds"]=int(d['rounds'])
    rows.append(r); print(json.dumps(r), flush=True)
json.dump(rows, open('profiles/priority_colour_counts.json','w'), indent=1)
