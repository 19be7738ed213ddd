#!/usr/bin/env python3
"""Nearest preceding symbol (nm -C, dynamic + static tables) of file offsets in a stripped library:
tools/nearest_symbol.py <lib.so> <hex offset> ... (used for profiles/r06/brunet/README.txt)."""
import subprocess,sys,bisect
lib=sys.argv[1]
syms=[]
for flag in (['-D'],[]):
    out=subprocess.run(['nm','-C','--defined-only',*flag,lib],capture_output=True,text=True).stdout
    for l in out.splitlines():
        p=l.split(' ',2)
        if len(p)==3 and p[1] in 'tTwWiI':
            syms.append((int(p[0],16),p[2]))
syms.sort()
addrs=[s[0] for s in syms]
for a in sys.argv[2:]:
    a=int(a,16); i=bisect.bisect_right(addrs,a)-1
    print(hex(a), (syms[i][1][:150], hex(a-syms[i][0])) if i>=0 else '?')
