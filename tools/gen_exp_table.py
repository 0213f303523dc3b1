"""Regenerates the constants of mcmc_clv_model_amd/csrc/fastmath.h (2^(j/64) table, ln2/64 split)."""
import math
from decimal import Decimal, getcontext

getcontext().prec = 80
ln2 = Decimal(2).ln()
L = ln2 / 64
m, e = math.frexp(float(L))
hi40 = math.ldexp(round(m * 2 ** 40), e - 40)
print("EXP_INV_L", float(Decimal(64) / ln2).hex())
print("EXP_L_HI", hi40.hex(), "EXP_L_LO", float(L - Decimal(hi40)).hex())
print([float(Decimal(2) ** (Decimal(j) / 64)).hex() for j in range(64)])
