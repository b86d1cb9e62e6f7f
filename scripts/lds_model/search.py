import sys; sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from bwd import analyze
cases = ((16,1,24),(16,1,16),(16,1,20),(32,1,16),(32,1,32),(32,1,24))
def total(**kw):
    t = 0
    for H,KX,Din in cases:
        r = analyze(H,KX,Din,**kw); t += sum(c for c,i in r.values())
    return t
def part(prefix, **kw):
    t = 0
    for H,KX,Din in cases:
        r = analyze(H,KX,Din,**kw); t += sum(c for k,(c,i) in r.items() if k.startswith(prefix))
    return t
print("baseline total", total())
for T in (False, True):
    for P in (32,33,34,36,40,17,18,20,24,28):
        if T and P < 32: pass
        if not T and P < 32: continue
        print("dxs T=%s P=%d: %d" % (T, P, part("dxs", dxs_pitch=P, dxs_T=T)))
for z in (8,16,24,40):
    print("zs extra %d: %d" % (z, part("zs", zpitch_extra=z)))
for d in (4,8,12,20):
    print("dhs pad %d: %d" % (d, part("dhs", dhs_pad=d)))
for x in (8,16,24):
    print("xr pad %d: xrs %d  hr pad: hrs %d" % (x, part("xrs", xr_pad=x), part("hrs", hr_pad=x)))
