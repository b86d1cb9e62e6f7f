"""Search a chunk-XOR swizzle of the backward's dz tile (zs [16 sequences][4H] bf16): stores are 16-bit
(lane = (sequence col, quad): gate-unit g H + 4 w + quad), MFMA operand reads are 16-byte chunks
(gate-units 32 k + 8 quad .. + 7). address(col, e) = col P + ((e / 8) ^ f(col)) 8 + e % 8."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sim import cycles, ideal


def cost(H, P, f):
    G4 = 4 * H; NW = 16 * H // 64; KB = G4 // 32
    def addr(col, e):
        return 2 * (col * P + (((e // 8) ^ f(col)) % (P // 8)) * 8 + e % 8)
    c = i = 0
    for w in range(NW):
        for g in range(4):
            a = [addr(l & 15, g * H + 4 * w + (l >> 4)) for l in range(64)]
            c += cycles("w16", a); i += ideal("w16")
        for k in range(KB):
            a = [addr(l & 15, 32 * k + 8 * (l >> 4)) for l in range(64)]
            c += 2 * cycles("r128", a); i += 2 * ideal("r128")
    return c, i


if __name__ == "__main__":
    fs = {"none": lambda c: 0}
    for sh in range(4):
        for m in (1, 3, 7):
            fs[f"(c>>{sh})&{m}"] = (lambda sh, m: (lambda c: (c >> sh) & m))(sh, m)
    for H in (16, 32, 64):
        G4 = 4 * H
        best = []
        for extra in (0, 8, 16, 24, 32):
            P = G4 + extra
            for name, f in fs.items():
                # the swizzle must keep chunks inside the row's G4 / 8 data chunks
                if any(((e // 8) ^ f(c)) >= G4 // 8 for c in range(16) for e in range(0, G4, 8)):
                    continue
                cc, ii = cost(H, P, f)
                best.append((cc, extra, name, ii))
        best.sort()
        print(H, best[:6], "current(16,none):", [b for b in best if b[1] == 16 and b[2] == "none"])
