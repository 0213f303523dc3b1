"""Regenerates the constants of mcmc_clv_model_amd/csrc/fastmath.h (2^(j/256) table, ln2/256 split)."""
import math
from decimal import Decimal, getcontext

getcontext().prec = 80
ln2 = Decimal(2).ln()
L = ln2 / 256
m, e = math.frexp(float(L))
hi = math.ldexp(round(m * 2 ** 38), e - 38)
print("EXP_INV_L", float(Decimal(256) / ln2).hex())
print("EXP_L_HI", hi.hex(), "EXP_L_LO", float(L - Decimal(hi)).hex())
print([float(Decimal(2) ** (Decimal(j) / 256)).hex() for j in range(256)])
