import sys; sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
from sim import cycles, ideal
def analyze(H, KX, Din, zpitch_extra=8, dxs_pitch=None, dxs_T=False, dhs_pad=4, xr_pad=8, hr_pad=8):
    G4 = 4*H; NT = 16*H; NW = NT//64; KB = G4//32; KPH = ((H+31)//32)*32; KSH = KPH//32
    ZP = G4 + zpitch_extra  # bf16
    HP = H + dhs_pad
    res = {}
    def add(name, kind, fn, waves=range(NW), count=1):
        c = 0; i = 0
        for w in waves:
            addrs = [fn(w, l) for l in range(64)]
            c += cycles(kind, addrs); i += ideal(kind)
        res[name] = (c*count, i*count)
    # zs b16 stores: zs[col][g*H+u], u = 4w+quad
    for g in range(4):
        add(f"zs_st{g}", "w16", lambda w,l,g=g: 2*((l&15)*ZP + g*H + 4*w + (l>>4)))
    # dhs float4 store: gd=(tid%(16H/4))*4 -> [gd/H][gd%H]
    ngd = 16*H//4
    add("dhs_st", "w128", lambda w,l: 4*(((w*64+l)%ngd)*4//H*HP + ((w*64+l)%ngd)*4%H))
    add("dhs_rd", "r32", lambda w,l: 4*((l&15)*HP + 4*w + (l>>4)))
    for k in range(KB):
        add(f"zs_rd{k}", "r128", lambda w,l,k=k: 2*((l&15)*ZP + 32*k + 8*(l>>4)), count=1 + 1)  # serial + dx
    NXB = 2*KX
    DXP = dxs_pitch if dxs_pitch else 32*KX
    xbw = [w for w in range(NW) if w < NXB]
    for r in range(4):
        if dxs_T:
            add(f"dxs_st{r}", "w32", lambda w,l,r=r: 4*((16*w + 4*(l>>4) + r)*DXP + (l&15)), waves=xbw)
        else:
            add(f"dxs_st{r}", "w32", lambda w,l,r=r: 4*((l&15)*DXP + 16*w + 4*(l>>4) + r), waves=xbw)
    GR = 4; ngx = 16*Din//GR
    for q in range(GR):
        def f(w,l,q=q):
            gx = ((w*64+l) % ngx)*GR; s, k = gx//Din, gx%Din
            return 4*((k+q)*DXP + s) if dxs_T else 4*(s*DXP + k + q)
        add(f"dxs_rd{q}", "r32", f)
    # RG staging
    XG = max(1, 16*32*KX//NT)
    XRP = 32*KX + xr_pad; HRP = KPH + hr_pad
    for q in range(XG):
        def f(w,l,q=q):
            wxe = ((w*64+l)*XG) % (16*Din); s, k = wxe//Din, wxe%Din
            return 2*(s*XRP + k + q)
        add(f"xrs_st{q}", "w16", f)
    add("hrs_st", "w16", lambda w,l: 2*(((w*64+l)//H)*HRP + (w*64+l)%H))
    for s_ in range(KX):
        add(f"xrs_rd{s_}", "r128", lambda w,l,s_=s_: 2*((l&15)*XRP + 32*s_ + 8*(l>>4)))
    for s_ in range(KSH):
        add(f"hrs_rd{s_}", "r128", lambda w,l,s_=s_: 2*((l&15)*HRP + 32*s_ + 8*(l>>4)))
    return res
def show(res, title):
    tc = sum(c for c,i in res.values()); ti = sum(i for c,i in res.values())
    print(f"{title}: total {tc} cycles vs ideal {ti} (+{tc-ti})")
    for k,(c,i) in res.items():
        if c > i: print(f"   {k:10s} {c:4d} / {i}")
if __name__ == "__main__":
    for H, KX, Din in ((16,1,24),(16,1,16),(32,1,16),(32,1,32)):
        show(analyze(H,KX,Din), f"H={H} KX={KX} Din={Din} current")
