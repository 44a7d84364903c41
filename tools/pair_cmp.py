import json,sys
a=json.load(open(sys.argv[1])); b=json.load(open(sys.argv[2]))
for n in a:
    bad=[k for k in a[n] if a[n][k]!=b[n][k]]
    print(n, len(bad), "bad of", len(a[n]), bad[:4], [ (a[n][k], b[n][k]) for k in bad[:2]])
