#!/bin/bash
# Instruction count + registers of the Homing step kernels (device asm), no GPU needed.
# EXTRA=<flags> for a variant; LAYOUT=<n> restricts to one layout (default: all).
cd "$(dirname "$0")/../swarmacb-isaaclab_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off ${STEPFLAGS--fno-slp-vectorize} -DSWARM_MISSION_ID=${MISSION:-2} $EXTRA \
  -I../../build/obj/gen --cuda-device-only -S -o /tmp/cs.s swarm_mission.hip -Rpass-analysis=kernel-resource-usage 2> /tmp/cs_res.txt || exit 1
LAYOUT=${LAYOUT:-} python3 - <<'PY'
import os, re
s = open('/tmp/cs.s').read()
res = open('/tmp/cs_res.txt').read()
lay = os.environ.get('LAYOUT')
for name in re.findall(r'^(_ZN5swarm11step_kernelI\w+):', s, re.M):
    if 'Lb0ELi20E' not in name or not re.search(r'step_kernelILi\dELi0E', name):
        continue
    m = re.search(r'Li20ELi(\d+)ELb(\d)EEE', name)
    if lay and m.group(1) != lay:
        continue
    start = s.index(name + ':'); end = s.index('.Lfunc_end', start)
    body = [l for l in s[start:end].split('\n') if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;')]
    salu = sum(1 for l in body if re.match(r'\ts_', l))
    r = re.search(re.escape(name) + r'.*?VGPRs: (\d+).*?ScratchSize \[bytes/lane\]: (\d+).*?SGPRs Spill: (\d+).*?VGPRs Spill: (\d+)', res, re.S)
    print(f'layout {m.group(1)} replay {m.group(2)}: insts {len(body)} (s_* {salu})',
          'vgpr/scratch/sgpr-spill/vgpr-spill', r.groups() if r else None)
PY
