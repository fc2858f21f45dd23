"""Topology summary of a HIP graph debug dump (nodes by kind, edges, in/out degrees)."""
import collections
import re
import sys

txt = open(sys.argv[1]).read()
nodes = dict(re.findall(r'"?(\w+)"?\s*\[[^\]]*label="([^"]*)"', txt))
edges = re.findall(r'"?(\w+)"?\s*->\s*"?(\w+)"?', txt)
kinds = collections.Counter(v.split('\\n')[0].split(' ')[0][:40] for v in nodes.values())
indeg, outdeg = collections.Counter(), collections.Counter()
for a, b in edges:
    outdeg[a] += 1
    indeg[b] += 1
print('nodes', len(nodes), 'edges', len(edges))
print('kinds', kinds.most_common(12))
print('roots', sum(1 for n in nodes if indeg[n] == 0), 'leaves', sum(1 for n in nodes if outdeg[n] == 0))
print('fan-out>1', sum(1 for n in nodes if outdeg[n] > 1), 'fan-in>1', sum(1 for n in nodes if indeg[n] > 1))
for n in nodes:
    if outdeg[n] > 1 or indeg[n] > 1:
        print(' branch node', n, nodes[n][:160].replace('\\n', ' | '), 'in', indeg[n], 'out', outdeg[n])
        break
