"""Pitch / chunk-swizzle search for the WG backward's transposed bf16 images zT [4H][RP], xT [XR][RP],
hT [H][RP] (rows = gate-unit / channel / unit, columns = the tile's 16 sequences): 16-bit transposed
stores, 16-byte MFMA operand reads of rows 16 d + col, chunk (lane >> 4) & 1.
address(row, k) = row RP + ((k / 8) ^ f(row)) 8 + k % 8."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sim import cycles


def cost(H, KX, Din, RP, f):
    NT = 16 * H; NW = NT // 64
    XG = max(1, 16 * 32 * KX // NT)
    def ad(row, k):
        return 2 * (row * RP + ((k // 8) ^ f(row)) * 8 + k % 8)
    c = 0
    for w in range(NW):
        for g in range(4):
            c += cycles("w16", [ad(g * H + 4 * w + (l >> 4), l & 15) for l in range(64)])
        for q in range(XG):
            a = []
            for l in range(64):
                wxe = ((w * 64 + l) * XG) % (16 * Din)
                a.append(ad(wxe % Din + q, wxe // Din))
            c += cycles("w16", a)
        c += cycles("w16", [ad((w * 64 + l) % H, (w * 64 + l) // H) for l in range(64)])
        c += cycles("r128", [ad(16 * w + (l & 15), 8 * ((l >> 4) & 1)) for l in range(64)])
        for d in range((Din + 16) // 16):
            c += cycles("r128", [ad(16 * d + (l & 15), 8 * ((l >> 4) & 1)) for l in range(64)])
        for k in range(H // 16):
            c += cycles("r128", [ad(16 * k + (l & 15), 8 * ((l >> 4) & 1)) for l in range(64)])
    return c


if __name__ == "__main__":
    fs = {"none": lambda r: 0}
    for sh in range(5):
        fs[f"(r>>{sh})&1"] = (lambda sh: (lambda r: (r >> sh) & 1))(sh)
    res = []
    for RP in (24, 32, 40):
        for name, f in fs.items():
            tot = sum(cost(H, KX, Din, RP, f) for H, KX, Din in ((16, 1, 20), (16, 1, 16), (32, 1, 16), (32, 1, 32)))
            res.append((tot, RP, name))
    res.sort()
    print(res[:8])
    print("current:", [r for r in res if r[1] == 24 and r[2] == "none"])
