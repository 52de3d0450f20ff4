"""Search the XOR swizzle sw(r) of the c5 strip ring (16 rows x 64 bf16 columns, 16-B chunks):
phase 1's ds_read_b128 row reads must hit 16 distinct 16-B slots per conflict group, phase 2's
ds_read_b64_tr_b16 transposed reads 32 distinct 8-B slots per 32-lane half.  Default: lsqp4's
16x16x32 phase-2 read; --p5: lsqp5's 32x32x16 read (rows 8h + 4e + q, chunk 4(ct&1) + 2cg + p/2)."""
import itertools
import sys
G1=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G1+= [[x+32 for x in G1[0]],[x+32 for x in G1[1]]]
def ok(f):
    for s in range(16):
        for grp in G1:
            slots=set()
            for l in grp:
                i=l&15; g=l>>4
                cs=4*(s&1)+g
                p=cs^f[i]
                a=(s>>1)*2048+i*128+p*16
                slots.add((a//16)%16)
            if len(slots)!=16: return False
    if "--p5" in sys.argv:
        for ct in range(16):
            for e in (0, 1):
                for grp in (range(0, 32), range(32, 64)):
                    slots = set()
                    for l in grp:
                        h = l >> 5; cg = (l >> 4) & 1; q = (l >> 2) & 3; p = l & 3
                        r = 8 * h + 4 * e + q
                        ch = 4 * (ct & 1) + 2 * cg + (p >> 1)
                        a = (ct >> 1) * 2048 + r * 128 + (ch ^ f[r]) * 16 + 8 * (p & 1)
                        slots.add((a // 8) % 32)
                    if len(slots) != 32: return False
        return True
    for ct in range(32):
        for half in (0,1):
            for grp in (range(0,32),range(32,64)):
                slots=set()
                for l in grp:
                    g=l>>4; qq=(l>>2)&3; p4=l&3
                    r=8*(g&1)+qq+4*half
                    ch=2*(ct&3)+(p4>>1)
                    a=(ct>>2)*2048+r*128+(ch^f[r])*16+8*(p4&1)
                    slots.add((a//8)%32)
                if len(slots)!=32: return False
    return True
sols=[]
for M in itertools.product(range(8),repeat=4):
    f=[0]*16
    for r in range(16):
        v=0
        for b in range(4):
            if r>>b&1: v^=M[b]
        f[r]=v
    if ok(f): sols.append((M,f))
print(len(sols)); print(sols[:5])
