// Device interpreter for the condition/selector bytecode (plan.h). Java semantics, bit-exact:
//   null handling       CompareConditionExpressionExecutor.java:38-42 (null -> false),
//                       And/Or/NotConditionExpressionExecutor.java (null -> false / not null -> TRUE)
//   numeric promotion   executor/condition/compare/** (e.g. GreaterThanCompareConditionExpressionExecutorFloatLong:
//                       float compare; EqualCompareConditionExpressionExecutorFloatLong: double compare)
//   arithmetic          executor/math/** (int/long wrap, /,% by zero -> null, double % = fmod)
// The program is wave-uniform (one query per launch), so instruction fetch is scalar and the op switch never
// diverges; the evaluation stack lives in LDS, one column of STACK entries per lane (conflict-free stride).
// Build with -ffp-contract=off (a fused multiply-add would change float/double results vs the JVM) and
// -fhip-fp32-correctly-rounded-divide-sqrt: then + - * / are the IEEE round-to-nearest operations Java uses.
// The functions are host+device so the test-only host harness (tests/native) runs the same code.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "plan.h"

#define SDG_FN __host__ __device__ __forceinline__

namespace sdg {

SDG_FN float bits_f32(int64_t v) { return __builtin_bit_cast(float, (uint32_t)v); }
SDG_FN double bits_f64(int64_t v) { return __builtin_bit_cast(double, v); }
SDG_FN int64_t f32_bits(float f) { return (int64_t)__builtin_bit_cast(uint32_t, f); }
SDG_FN int64_t f64_bits(double d) { return __builtin_bit_cast(int64_t, d); }

// typed column load -> 64-bit payload (same encoding as sdg_out)
SDG_FN int64_t load_col(const void* col, uint8_t kind, int64_t row) {
    switch (kind) {
        case VK_I32: return (int64_t)((const int32_t*)col)[row];
        case VK_I64: return ((const int64_t*)col)[row];
        case VK_F32: return (int64_t)((const uint32_t*)col)[row];
        case VK_F64: return ((const int64_t*)col)[row];
        case VK_BOOL: return (int64_t)((const uint8_t*)col)[row];
        default: return (int64_t)((const uint32_t*)col)[row];
    }
}

SDG_FN int64_t cvt(int64_t v, uint8_t from, uint8_t to) {
    if (from == to) return v;
    switch (to) {
        case VK_I64: return (int64_t)(int32_t)v;  // only int -> long widens
        case VK_F32: return from == VK_I32 ? f32_bits((float)(int32_t)v) : f32_bits((float)v);
        case VK_F64:
            if (from == VK_I32) return f64_bits((double)(int32_t)v);
            if (from == VK_I64) return f64_bits((double)v);
            return f64_bits((double)bits_f32(v));
        default: return v;
    }
}

template <class T>
SDG_FN bool cmpT(uint8_t op, T a, T b) {
    switch (op) {
        case CMP_EQ: return a == b;
        case CMP_NE: return a != b;
        case CMP_GT: return a > b;
        case CMP_GE: return a >= b;
        case CMP_LT: return a < b;
        default: return a <= b;
    }
}

SDG_FN bool cmp(uint8_t op, uint8_t k, int64_t a, int64_t b) {
    switch (k) {
        case VK_I32: return cmpT<int32_t>(op, (int32_t)a, (int32_t)b);
        case VK_I64: return cmpT<int64_t>(op, a, b);
        case VK_F32: return cmpT<float>(op, bits_f32(a), bits_f32(b));
        case VK_F64: return cmpT<double>(op, bits_f64(a), bits_f64(b));
        case VK_BOOL: return cmpT<int>(op, (int)(a != 0), (int)(b != 0));
        default: return cmpT<uint32_t>(op, (uint32_t)a, (uint32_t)b);  // string ids: == / != only
    }
}

// returns false (and *null = true) when Java would produce null
SDG_FN int64_t arith(uint8_t op, uint8_t k, int64_t a, int64_t b, bool* null) {
    *null = false;
    switch (k) {
        case VK_I32: {
            int32_t x = (int32_t)a, y = (int32_t)b;
            uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
            switch (op) {
                case AR_ADD: return (int64_t)(int32_t)(ux + uy);
                case AR_SUB: return (int64_t)(int32_t)(ux - uy);
                case AR_MUL: return (int64_t)(int32_t)(ux * uy);
                case AR_DIV:
                    if (y == 0) { *null = true; return 0; }
                    if (x == INT32_MIN && y == -1) return x;
                    return (int64_t)(x / y);
                default:
                    if (y == 0) { *null = true; return 0; }
                    if (y == -1) return 0;
                    return (int64_t)(x % y);
            }
        }
        case VK_I64: {
            uint64_t ux = (uint64_t)a, uy = (uint64_t)b;
            switch (op) {
                case AR_ADD: return (int64_t)(ux + uy);
                case AR_SUB: return (int64_t)(ux - uy);
                case AR_MUL: return (int64_t)(ux * uy);
                case AR_DIV:
                    if (b == 0) { *null = true; return 0; }
                    if (a == INT64_MIN && b == -1) return a;
                    return a / b;
                default:
                    if (b == 0) { *null = true; return 0; }
                    if (b == -1) return 0;
                    return a % b;
            }
        }
        case VK_F32: {
            float x = bits_f32(a), y = bits_f32(b);
            switch (op) {
                case AR_ADD: return f32_bits(x + y);
                case AR_SUB: return f32_bits(x - y);
                case AR_MUL: return f32_bits(x * y);
                case AR_DIV:
                    if (y == 0.0f) { *null = true; return 0; }
                    return f32_bits(x / y);
                default:
                    if (y == 0.0f) { *null = true; return 0; }
                    return f32_bits(fmodf(x, y));
            }
        }
        default: {
            double x = bits_f64(a), y = bits_f64(b);
            switch (op) {
                case AR_ADD: return f64_bits(x + y);
                case AR_SUB: return f64_bits(x - y);
                case AR_MUL: return f64_bits(x * y);
                case AR_DIV:
                    if (y == 0.0) { *null = true; return 0; }
                    return f64_bits(x / y);
                default:
                    if (y == 0.0) { *null = true; return 0; }
                    return f64_bits(fmod(x, y));
            }
        }
    }
}

// Acc must provide:
//   void load(int slot, int col, int chain, uint8_t kind, int64_t* v, bool* null);
//   bool slot_empty(int slot, int chain);
//   void agg(int g, int64_t* v, bool* null);   (selector post pass; never reached elsewhere)
// stk: this lane's LDS stack base, entries at stk[i * stride]
template <class Acc>
SDG_FN void run(const Instr* __restrict__ code, Prog p, const int64_t* __restrict__ consts,
                                    Acc& acc, int64_t* stk, int stride, int64_t* out, bool* out_null) {
    uint32_t nulls = 0;
    int sp = 0;
    for (int pc = p.start; pc < p.start + p.len; ++pc) {
        const Instr in = code[pc];
        switch (in.op) {
            case OP_LOAD: {
                int64_t v;
                bool n;
                acc.load(in.a, in.b, in.c, in.k, &v, &n);
                stk[sp * stride] = v;
                nulls = n ? (nulls | (1u << sp)) : (nulls & ~(1u << sp));
                ++sp;
                break;
            }
            case OP_CONST:
                stk[sp * stride] = consts[in.imm];
                nulls &= ~(1u << sp);
                ++sp;
                break;
            case OP_CVT:
                if (!(nulls & (1u << (sp - 1)))) stk[(sp - 1) * stride] = cvt(stk[(sp - 1) * stride], in.a, in.k);
                break;
            case OP_CMP: {
                bool na = nulls & (1u << (sp - 2)), nb = nulls & (1u << (sp - 1));
                int64_t a = stk[(sp - 2) * stride], b = stk[(sp - 1) * stride];
                bool r = !(na || nb) && cmp(in.a, in.k, a, b);
                --sp;
                stk[(sp - 1) * stride] = r;
                nulls &= ~(3u << (sp - 1));
                break;
            }
            case OP_ARITH: {
                bool na = nulls & (1u << (sp - 2)), nb = nulls & (1u << (sp - 1));
                int64_t a = stk[(sp - 2) * stride], b = stk[(sp - 1) * stride];
                --sp;
                nulls &= ~(3u << (sp - 1));
                if (na || nb) {
                    nulls |= 1u << (sp - 1);
                } else {
                    bool n;
                    int64_t r = arith(in.a, in.k, a, b, &n);
                    stk[(sp - 1) * stride] = r;
                    if (n) nulls |= 1u << (sp - 1);
                }
                break;
            }
            case OP_AND:
            case OP_OR: {
                bool ta = !(nulls & (1u << (sp - 2))) && stk[(sp - 2) * stride] != 0;
                bool tb = !(nulls & (1u << (sp - 1))) && stk[(sp - 1) * stride] != 0;
                --sp;
                stk[(sp - 1) * stride] = in.op == OP_AND ? (ta && tb) : (ta || tb);
                nulls &= ~(3u << (sp - 1));
                break;
            }
            case OP_NOT: {
                bool t = !(nulls & (1u << (sp - 1))) && stk[(sp - 1) * stride] != 0;
                stk[(sp - 1) * stride] = !t;
                nulls &= ~(1u << (sp - 1));
                break;
            }
            case OP_ISNULL: {
                bool n = nulls & (1u << (sp - 1));
                stk[(sp - 1) * stride] = n;
                nulls &= ~(1u << (sp - 1));
                break;
            }
            case OP_SLOTNULL:
                stk[sp * stride] = acc.slot_empty(in.a, in.c);
                nulls &= ~(1u << sp);
                ++sp;
                break;
            case OP_COND: {
                bool n = nulls & (1u << (sp - 1));
                if (n) stk[(sp - 1) * stride] = 0;
                nulls &= ~(1u << (sp - 1));
                break;
            }
            case OP_IFELSE: {  // IfThenElseFunctionExecutor: Boolean.TRUE.equals(cond) ? then : else
                const int b0 = sp - 3;
                const bool c = !(nulls & (1u << b0)) && stk[b0 * stride] != 0;
                const int pick = c ? b0 + 1 : b0 + 2;
                const int64_t v = stk[pick * stride];
                const bool n = nulls & (1u << pick);
                stk[b0 * stride] = v;
                nulls = (nulls & ~(7u << b0)) | (n ? 1u << b0 : 0u);
                sp = b0 + 1;
                break;
            }
            case OP_COALESCE: {  // the first non-null argument
                const int na = in.a, b0 = sp - na;
                int64_t v = 0;
                bool n = true;
                for (int i = 0; i < na && n; ++i)
                    if (!(nulls & (1u << (b0 + i)))) {
                        v = stk[(b0 + i) * stride];
                        n = false;
                    }
                stk[b0 * stride] = v;
                nulls = (nulls & ~(((1u << na) - 1u) << b0)) | (n ? 1u << b0 : 0u);
                sp = b0 + 1;
                break;
            }
            case OP_MAXMIN: {  // Maximum/MinimumFunctionExecutor.execute(Object[]) (one argument: returned as is)
                const int na = in.a, b0 = sp - na;
                if (na > 1) {
                    const bool mx = in.c != 0;
                    const double start = mx ? 4.9406564584124654e-324 : 1.7976931348623157e308;
                    double best = start;
                    for (int i = 0; i < na; ++i) {
                        const int64_t r = stk[(b0 + i) * stride];
                        double x = start;
                        if (!(nulls & (1u << (b0 + i))))
                            x = in.k == VK_I32 ? (double)(int32_t)r : in.k == VK_I64 ? (double)r
                                : in.k == VK_F32 ? (double)bits_f32(r) : bits_f64(r);
                        if (mx ? x > best : x < best) best = x;
                    }
                    int64_t v;
                    if (in.k == VK_I32) v = best >= 2147483647.0 ? INT32_MAX : best <= -2147483648.0 ? INT32_MIN : (int64_t)(int32_t)best;
                    else if (in.k == VK_I64) v = best >= 9223372036854775807.0 ? INT64_MAX : best <= -9223372036854775808.0 ? INT64_MIN : (int64_t)best;
                    else if (in.k == VK_F32) v = f32_bits((float)best);
                    else v = f64_bits(best);
                    stk[b0 * stride] = v;
                    nulls &= ~(((1u << na) - 1u) << b0);
                    sp = b0 + 1;
                }
                break;
            }
            case OP_SLOTLEN: {  // MultiValueVariableFunctionExecutor's list size (ExpressionParser.java:1430-1436)
                int n = 0;
                while (n < in.c && !acc.slot_empty(in.a, n)) ++n;
                stk[sp * stride] = n;
                nulls &= ~(1u << sp);
                ++sp;
                break;
            }
            case OP_AGG: {
                int64_t v;
                bool n;
                acc.agg(in.a, &v, &n);
                stk[sp * stride] = v;
                nulls = n ? (nulls | (1u << sp)) : (nulls & ~(1u << sp));
                ++sp;
                break;
            }
            case OP_JAND:
            case OP_JOR: {
                const bool t = !(nulls & (1u << (sp - 1))) && stk[(sp - 1) * stride] != 0;
                if (t == (in.op == OP_JOR)) {
                    stk[(sp - 1) * stride] = t;
                    nulls &= ~(1u << (sp - 1));
                    pc += in.imm - 1;
                }
                break;
            }
            default:
                break;
        }
    }
    *out = stk[0];
    *out_null = (nulls & 1u) != 0;
}

// FastPred evaluation (compile-time recognised `a OP b`): identical results to the bytecode
template <class Acc>
SDG_FN bool fast_pass(const FastPred& f, Acc& acc) {
    int64_t a, b;
    bool na, nb;
    acc.load(f.sa, f.ca, f.ia, f.ka, &a, &na);
    if (na) return false;
    a = cvt(a, f.ka, f.t);
    if (f.kind == FP_CONST) {
        b = f.konst;
    } else {
        acc.load(f.sb, f.cb, f.ib, f.kb, &b, &nb);
        if (nb) return false;
        b = cvt(b, f.kb, f.t);
    }
    return cmp(f.op, f.t, a, b);
}

// a filter passes iff its result is non-null and true (FilterProcessor.java:48-60)
template <class Acc>
SDG_FN bool pass(const Instr* code, Prog p, const int64_t* consts, Acc& acc, int64_t* stk,
                                     int stride) {
    if (p.len == 0) return true;
    int64_t v;
    bool n;
    run(code, p, consts, acc, stk, stride, &v, &n);
    return !n && v != 0;
}

}  // namespace sdg
