// fe_vm.h -- the final-exponentiation step machine's interpreter loop (kernels.h
// "Fq12 step machine"), shared by k_fq12_vm (kernels_fe.hip) and the one-pass
// k_pairing_full (kernels_pairing.hip).  Included inside namespace bn by a
// BN_SPLIT translation unit after kernels.h.
#pragma once

namespace bn {

__device__ __forceinline__ uint32_t* vm_slot_ptr(uint32_t* slots, size_t nl, uint32_t s) {
    return slots + (size_t)s * kSlotLaneWords * nl;
}
// Runs the program on lane i's element (lane-strided slots, `lanes` lanes in
// all); returns the last step's result.  Balance positions are pos_base +
// step * 256 + squarings done in the step.  store_last = false: the last
// step's result is only returned (k_pairing_full writes the Gt itself).
__device__ __forceinline__ Fq12<kF> fq12_vm_run(const uint32_t* __restrict__ prog, int nsteps, uint32_t* slots,
                                               size_t lanes, size_t i, const Balance& bal, uint32_t pos_base,
                                               bool store_last) {
    Fq12<kF> acc = widen<kF>(fq12_one());  // the previous step's result, kept in registers
#pragma unroll 1
    for (int pc = 0; pc < nsteps; ++pc) {
        const uint32_t ins = prog[2 * pc];  // uniform: scalar loads
        const uint32_t aux = prog[2 * pc + 1];
        const uint32_t op = ins & 0xff, k = aux & 0xff, flags = aux >> 8;
        // The slot stride passes through an empty asm once per step, so the
        // word offsets of a lane-strided Fq12 (w * nl, uniform) are rebuilt where
        // they are used instead of being hoisted out of the step loop, where they
        // would occupy ~216 SGPRs and spill through VGPR lanes.
        size_t nn = lanes;
        asm volatile("" : "+s"(nn));
        uint32_t* d = vm_slot_ptr(slots, nn, (ins >> 8) & 0xff);
        const uint32_t* a = vm_slot_ptr(slots, nn, (ins >> 16) & 0xff);
        const uint32_t* b = vm_slot_ptr(slots, nn, ins >> 24);
        const uint32_t pos = pos_base + ((uint32_t)pc << 8);
        balance_step(bal, pos);
        Fq12<kF> x;
        if (flags & kFlagAccA) x = acc; else x = ld_fq12_buf<kF>(a, nn, i);
        Fq12<kF> r;
        switch (op) {
            case OP_MOV: r = x; break;
            case OP_MUL: {
                // (the operand loaded before the squarings instead: more scratch, within
                // noise, profiles/r3v_ab_vm_preload.txt)
#pragma unroll 1
                for (uint32_t j = 0; j < k; ++j) {
                    balance_step(bal, pos | j);
                    x = cyc_sqr(x);
                }
                balance_step(bal, pos | 255u);
                Fq12<kF> y = ld_fq12_buf<kF>(b, nn, i);
                if (flags & kFlagConjB) y = fq12_conj(y);
                r = mul12(x, y);
                if (flags & kFlagConjOut) r = fq12_conj(r);
                break;
            }
            case OP_SQR: r = narrow12<kF>(fq12_sqr(x)); break;
            case OP_CYC: {
#pragma unroll 1
                for (uint32_t j = 0; j < k; ++j) {
                    balance_step(bal, pos | j);
                    x = cyc_sqr(x);
                }
                r = x;
                break;
            }
            case OP_CONJ: r = fq12_conj(x); break;
            case OP_FROB1: r = narrow12<kF>(fq12_frobenius_map<1>(x)); break;
            case OP_FROB2: r = narrow12<kF>(fq12_frobenius_map<2>(x)); break;
            case OP_FROB3: r = narrow12<kF>(fq12_frobenius_map<3>(x)); break;
            default: r = narrow12<kF>(fq12_inv(x)); break;  // OP_INV
        }
        acc = r;
        if (!(flags & kFlagNoStore) && (store_last || pc + 1 < nsteps)) st_fq12_buf(d, nn, i, r);
    }
    return acc;
}

}  // namespace bn
