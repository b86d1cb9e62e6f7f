import sys; sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from sim import cycles, ideal
def analyze(H, KX, Din, RP=24):
    G4 = 4*H; NT = 16*H; NW = NT//64
    res = {}
    def add(name, kind, fn, waves=range(NW)):
        c = i = 0
        for w in waves:
            c += cycles(kind, [fn(w,l) for l in range(64)]); i += ideal(kind)
        res[name] = (c, i)
    for g in range(4):
        add(f"zT_st{g}", "w16", lambda w,l,g=g: 2*((g*H + 4*w + (l>>4))*RP + (l&15)))
    XG = max(1, 16*32*KX//NT)
    for q in range(XG):
        def f(w,l,q=q):
            wxe = ((w*64+l)*XG) % (16*Din); s, k = wxe//Din, wxe%Din
            return 2*((k+q)*RP + s)
        add(f"xT_st{q}", "w16", f)
    add("hT_st", "w16", lambda w,l: 2*(((w*64+l)%H)*RP + (w*64+l)//H))
    add("zT_rd", "r128", lambda w,l: 2*((16*w + (l&15))*RP + 8*((l>>4)&1)))
    dtw = (Din+16)//16
    for d in range(dtw):
        add(f"xT_rd{d}", "r128", lambda w,l,d=d: 2*((16*d + (l&15))*RP + 8*((l>>4)&1)))
    for k in range(H//16):
        add(f"hT_rd{k}", "r128", lambda w,l,k=k: 2*((16*k + (l&15))*RP + 8*((l>>4)&1)))
    return res
for RP in (24, 40, 56, 20, 28, 36):
    t = 0; ti = 0; det = {}
    for H,KX,Din in ((16,1,20),(16,1,16),(32,1,16),(32,1,32)):
        r = analyze(H,KX,Din,RP)
        for k,(c,i) in r.items():
            t += c; ti += i; det[k[:3]] = det.get(k[:3],0) + c - i
    print(RP, t, ti, det)
