/* jit_blob.S — the code-object templates of the tree compiler (jit.cpp),
 * built from jit_template.hip with 1 MiB and 8 MiB code areas, and of the
 * Float64 tree compiler (jit64.cpp, jit64_template.hip, 4 MiB), embedded in
 * libsrhip.so as read-only data. */
    .section .rodata
    .balign 64
    .globl srhip_jit_tmpl_s
srhip_jit_tmpl_s:
    .incbin "gen/jit_tmpl_s.hsaco"
    .globl srhip_jit_tmpl_s_end
srhip_jit_tmpl_s_end:
    .balign 64
    .globl srhip_jit_tmpl_l
srhip_jit_tmpl_l:
    .incbin "gen/jit_tmpl_l.hsaco"
    .globl srhip_jit_tmpl_l_end
srhip_jit_tmpl_l_end:
    .balign 64
    .globl srhip_jit64_tmpl
srhip_jit64_tmpl:
    .incbin "gen/jit64_tmpl.hsaco"
    .globl srhip_jit64_tmpl_end
srhip_jit64_tmpl_end:
    .section .note.GNU-stack,"",@progbits
