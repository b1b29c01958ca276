"""Identifiers of include/srhip.h (checked against the header by
tests/test_abi.py)."""

F32, F64 = 0, 1
PROGRAM_VARYING_CONSTANTS = 1  # srhip_program_create_ex flag (include/srhip.h)
PROGRAM_INTERPRETED = 2  # srhip_program_create_ex flag: no loss / output tree code (include/srhip.h)
X_JULIA, X_FEATURE_MAJOR = 0, 1
NODE_CONST, NODE_FEATURE, NODE_UNARY, NODE_BINARY = 0, 1, 2, 3

BOPS = ["ADD", "SUB", "MUL", "DIV", "POW", "GREATER", "LOGICAL_OR", "LOGICAL_AND", "MOD", "MAX", "MIN"]
UOPS = ["NEG", "SQUARE", "CUBE", "EXP", "ABS", "LOG", "LOG2", "LOG10", "LOG1P", "SQRT", "SIN", "COS",
        "TAN", "SINH", "COSH", "TANH", "ATAN", "ASINH", "ACOSH", "ATANH_CLIP", "ERF", "ERFC", "GAMMA",
        "RELU", "ROUND", "FLOOR", "CEIL", "SIGN", "INV"]
BOP = {n: i for i, n in enumerate(BOPS)}
UOP = {n: i for i, n in enumerate(UOPS)}

LOSSES = ["L2", "L1", "LP", "HUBER", "LOGCOSH", "L1EPSINS", "L2EPSINS", "QUANTILE", "PERIODIC",
          "LOGITDIST", "LPINT"]
LOSS = {n: i for i, n in enumerate(LOSSES)}

# Julia operator names → (arity, id), applying binopmap / unaopmap
# (src/Options.jl:86-120). Mirrors srhip_op_lookup.
OP_NAMES = {
    "+": (2, BOP["ADD"]), "plus": (2, BOP["ADD"]),
    "-": (2, BOP["SUB"]), "sub": (2, BOP["SUB"]),
    "*": (2, BOP["MUL"]), "mult": (2, BOP["MUL"]),
    "/": (2, BOP["DIV"]), "div": (2, BOP["DIV"]),
    "^": (2, BOP["POW"]), "pow": (2, BOP["POW"]), "safe_pow": (2, BOP["POW"]),
    "greater": (2, BOP["GREATER"]), "logical_or": (2, BOP["LOGICAL_OR"]),
    "logical_and": (2, BOP["LOGICAL_AND"]), "mod": (2, BOP["MOD"]),
    "max": (2, BOP["MAX"]), "min": (2, BOP["MIN"]),
    "neg": (1, UOP["NEG"]), "square": (1, UOP["SQUARE"]), "cube": (1, UOP["CUBE"]),
    "exp": (1, UOP["EXP"]), "abs": (1, UOP["ABS"]),
    "log": (1, UOP["LOG"]), "safe_log": (1, UOP["LOG"]),
    "log2": (1, UOP["LOG2"]), "safe_log2": (1, UOP["LOG2"]),
    "log10": (1, UOP["LOG10"]), "safe_log10": (1, UOP["LOG10"]),
    "log1p": (1, UOP["LOG1P"]), "safe_log1p": (1, UOP["LOG1P"]),
    "sqrt": (1, UOP["SQRT"]), "safe_sqrt": (1, UOP["SQRT"]),
    "sin": (1, UOP["SIN"]), "cos": (1, UOP["COS"]), "tan": (1, UOP["TAN"]),
    "sinh": (1, UOP["SINH"]), "cosh": (1, UOP["COSH"]), "tanh": (1, UOP["TANH"]),
    "atan": (1, UOP["ATAN"]), "asinh": (1, UOP["ASINH"]),
    "acosh": (1, UOP["ACOSH"]), "safe_acosh": (1, UOP["ACOSH"]),
    "atanh": (1, UOP["ATANH_CLIP"]), "atanh_clip": (1, UOP["ATANH_CLIP"]),
    "erf": (1, UOP["ERF"]), "erfc": (1, UOP["ERFC"]), "gamma": (1, UOP["GAMMA"]),
    "relu": (1, UOP["RELU"]), "round": (1, UOP["ROUND"]), "floor": (1, UOP["FLOOR"]),
    "ceil": (1, UOP["CEIL"]), "sign": (1, UOP["SIGN"]), "inv": (1, UOP["INV"]),
}
