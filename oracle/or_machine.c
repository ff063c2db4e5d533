/*
 * ORACLE — test infrastructure only.
 *
 * CPU restatement of:
 *   - Program::from            crates/core/executor/src/program.rs:22-45
 *   - Executor::run / execute_* / rr_traced / rw_traced
 *                              crates/core/executor/src/executor.rs:71-326
 *     NORMAL FORM: the reference drains a randomly-seeded hashbrown map into
 *     record.cpu_memory_access (executor.rs:74-76); here memory events are SORTED BY ADDR.
 *   - per-chip generate_trace / generate_dependencies (files cited per function)
 *   - the lookups each chip's eval() emits (sends then receives, emission order)
 *   - the AIR constraints of each chip's eval(), in emission order, folded as
 *     acc = acc*alpha + c (crates/stark/src/folder.rs:68-72), followed by the LogUp
 *     constraints of eval_permutation_constraints (crates/stark/src/permutation.rs:157-272).
 */
#include <stdlib.h>
#include <string.h>
#include "or_machine.h"

const or_chip_info OR_CHIPS[NUM_CHIPS] = {
    {"Cpu", 31, 0, 0},      {"Program", 1, 6, 0}, {"AddSub", 7, 0, 1},
    {"Jump", 45, 0, 1},     {"Memory", 12, 0, 0}, {"Byte", 2, 2, 0},
    {"MemoryInstrs", 41, 0, 0}, {"IO", 5, 0, 1},
};

/* ---------------------------------------------------------------- program.rs:22-45 */
int or_parse_program(const char* src, or_program* p) {
  size_t cap = strlen(src) + 1, n = 0, sp = 0;
  p->ins = malloc(sizeof(or_instr) * cap);
  size_t* stack = malloc(sizeof(size_t) * cap);
  for (const char* c = src; *c; c++) {
    int op;
    switch (*c) {
      case '>': op = OP_FWD; break;
      case '<': op = OP_BWD; break;
      case '+': op = OP_ADD; break;
      case '-': op = OP_SUB; break;
      case '.': op = OP_OUTPUT; break;
      case ',': op = OP_INPUT; break;
      case '[': op = OP_LOOP_START; break;
      case ']': op = OP_LOOP_END; break;
      case ' ': case '\n': case '\r': continue;
      default: free(stack); return -1; /* reference: unreachable!() */
    }
    if (op == OP_LOOP_START) {
      p->ins[n].opcode = op; p->ins[n].op_a = 0;
      stack[sp++] = n++;
    } else if (op == OP_LOOP_END) {
      if (!sp) { free(stack); return -2; }
      size_t start = stack[--sp];
      p->ins[start].op_a = (uint32_t)n;
      p->ins[n].opcode = op; p->ins[n].op_a = (uint32_t)(start + 1);
      n++;
    } else {
      p->ins[n].opcode = op; p->ins[n].op_a = 0; n++;
    }
  }
  free(stack);
  p->n = n;
  return 0;
}

/* ------------------------------------------------------------------ memory map */
typedef struct { uint32_t key; uint32_t ts; uint8_t val; uint8_t used; int64_t ev; } slot;
typedef struct { slot* s; size_t cap, n; } memmap;
static void mm_init(memmap* m) { m->cap = 1024; m->n = 0; m->s = calloc(m->cap, sizeof(slot)); }
static slot* mm_get(memmap* m, uint32_t k);
static void mm_grow(memmap* m) {
  slot* old = m->s; size_t oc = m->cap;
  m->cap *= 2; m->s = calloc(m->cap, sizeof(slot)); m->n = 0;
  for (size_t i = 0; i < oc; i++) if (old[i].used) { slot* d = mm_get(m, old[i].key); *d = old[i]; }
  free(old);
}
static slot* mm_get(memmap* m, uint32_t k) {
  if (m->n * 2 >= m->cap) mm_grow(m);
  size_t h = ((uint64_t)k * 0x9E3779B97F4A7C15ull) >> 20;
  for (size_t i = h & (m->cap - 1);; i = (i + 1) & (m->cap - 1)) {
    if (!m->s[i].used) {
      m->s[i].used = 1; m->s[i].key = k; m->s[i].ts = 0; m->s[i].val = 0; m->s[i].ev = -1;
      m->n++;
      return &m->s[i];
    }
    if (m->s[i].key == k) return &m->s[i];
  }
}

#define PUSH(arr, n, cap, T) do { if ((n) == (cap)) { (cap) = (cap) ? 2 * (cap) : 1024; \
  arr = realloc(arr, sizeof(T) * (cap)); } } while (0)

static int cmp_mem(const void* a, const void* b) {
  const or_mem_ev* x = a; const or_mem_ev* y = b;
  return x->addr < y->addr ? -1 : (x->addr > y->addr);
}

/* ---------------------------------------------------------- executor.rs:71-326 */
int or_execute(const or_program* p, const uint8_t* in, size_t nin, or_record* r) {
  memset(r, 0, sizeof *r);
  r->prog = *p;
  size_t cap_cpu = 0, cap_alu = 0, cap_j = 0, cap_mi = 0, cap_io = 0, cap_mem = 0, cap_out = 0;
  memmap mm; mm_init(&mm);
  uint32_t pc = 0, mp = 0, clk = 0;
  size_t inptr = 0;
  uint64_t gclk = 0;
  int err = 0;
  if (p->n == 0) { err = -3; goto done; }
  for (;;) {
    or_instr ins = p->ins[pc];
    uint32_t next_pc = pc + 1, jmp_dst = 0;
    uint8_t next_mv = 0, mv = 0;
    uint32_t mp0 = mp;
    or_memacc acc_mv = {0}, acc_next = {0};
    /* rr_traced / rw_traced */
#define TRACE_ACCESS(ADDR, TS, WRITE, VAL, OUTREC) do { \
      slot* sl = mm_get(&mm, (ADDR)); \
      uint8_t pv = sl->val; uint32_t pts = sl->ts; \
      if (WRITE) sl->val = (VAL); \
      sl->ts = (TS); \
      if (sl->ev < 0) { PUSH(r->mem, r->nmem, cap_mem, or_mem_ev); \
        r->mem[r->nmem].addr = (ADDR); r->mem[r->nmem].init_ts = pts; r->mem[r->nmem].init_v = pv; \
        sl->ev = (int64_t)r->nmem++; } \
      r->mem[sl->ev].final_ts = sl->ts; r->mem[sl->ev].final_v = sl->val; \
      (OUTREC).kind = (WRITE) ? 2 : 1; (OUTREC).value = sl->val; (OUTREC).ts = sl->ts; \
      (OUTREC).prev_value = pv; (OUTREC).prev_ts = pts; } while (0)
    switch (ins.opcode) {
      case OP_FWD: mp = mp + 1; break;
      case OP_BWD: mp = mp - 1; break;
      case OP_ADD: case OP_SUB: {
        TRACE_ACCESS(mp, clk + 1, 0, 0, acc_mv);
        mv = acc_mv.value;
        next_mv = ins.opcode == OP_ADD ? (uint8_t)(mv + 1) : (uint8_t)(mv - 1);
        TRACE_ACCESS(mp, clk + 2, 1, next_mv, acc_next);
        break;
      }
      case OP_LOOP_START: case OP_LOOP_END: {
        TRACE_ACCESS(mp, clk + 1, 0, 0, acc_mv);
        mv = acc_mv.value;
        if (ins.opcode == OP_LOOP_START) next_pc = mv == 0 ? ins.op_a : pc + 1;
        else next_pc = mv != 0 ? ins.op_a : pc + 1;
        jmp_dst = next_pc;
        break;
      }
      case OP_INPUT: {
        if (inptr >= nin) { err = -4; goto done; }
        uint8_t v = in[inptr];
        TRACE_ACCESS(mp, clk + 1, 1, v, acc_mv);
        mv = v;
        break;
      }
      case OP_OUTPUT: {
        TRACE_ACCESS(mp, clk + 1, 0, 0, acc_mv);
        mv = acc_mv.value;
        PUSH(r->output, r->noutput, cap_out, uint8_t);
        r->output[r->noutput++] = mv;
        break;
      }
    }
    /* emit_events (executor.rs:178-239) */
    PUSH(r->cpu, r->ncpu, cap_cpu, or_cpu_ev);
    or_cpu_ev* ce = &r->cpu[r->ncpu++];
    ce->clk = clk; ce->pc = pc; ce->next_pc = next_pc; ce->mp = mp0; ce->next_mp = mp;
    ce->mv = mv; ce->next_mv = next_mv; ce->mv_access = acc_mv; ce->next_mv_access = acc_next;
    if (ins.opcode == OP_ADD || ins.opcode == OP_SUB) {
      PUSH(r->alu, r->nalu, cap_alu, or_alu_ev);
      or_alu_ev e = {pc, ins.opcode, next_mv, mv}; r->alu[r->nalu++] = e;
    }
    if (ins.opcode == OP_LOOP_START || ins.opcode == OP_LOOP_END) {
      PUSH(r->jump, r->njump, cap_j, or_jump_ev);
      or_jump_ev e = {pc, next_pc, ins.opcode, jmp_dst, mv}; r->jump[r->njump++] = e;
    }
    if (ins.opcode == OP_FWD || ins.opcode == OP_BWD) {
      PUSH(r->mi, r->nmi, cap_mi, or_meminstr_ev);
      or_meminstr_ev e = {clk, pc, ins.opcode, mp0, mp}; r->mi[r->nmi++] = e;
    }
    if (ins.opcode == OP_INPUT || ins.opcode == OP_OUTPUT) {
      PUSH(r->io, r->nio, cap_io, or_io_ev);
      or_io_ev e = {pc, ins.opcode, mp0, mv}; r->io[r->nio++] = e;
    }
    pc = next_pc;
    clk += 2;
    gclk++;
    if (pc == p->n) break;
  }
done:
  free(mm.s);
  qsort(r->mem, r->nmem, sizeof(or_mem_ev), cmp_mem);
  r->global_clk = gclk;
  r->final_pc = pc;
  r->final_mp = mp;
  return err;
}

/* Byte-lookup multiplicities: CpuChip::generate_dependencies (cpu/trace.rs:58-79,
 * event_to_row :88-150 incl. populate_clk and MemoryAccessCols::populate_access
 * memory/consistency/trace.rs:52-77) and AddSubChip (alu/mod.rs:95-116, AddOperation::
 * populate operations/add.rs:20-40).  Jump/MemoryInstrs traces emit none. */
void or_generate_dependencies(or_record* r) {
  r->u8_mult = calloc(256, sizeof(uint64_t));
  r->u16_mult = calloc(65536, sizeof(uint64_t));
  for (size_t i = 0; i < r->ncpu; i++) {
    const or_cpu_ev* e = &r->cpu[i];
    r->u16_mult[e->clk & 0xffff]++;
    r->u8_mult[(e->clk >> 16) & 0xff]++;
    if (e->mv_access.kind) {
      uint32_t d = e->mv_access.ts - e->mv_access.prev_ts - 1;
      r->u16_mult[d & 0xffff]++;
      r->u8_mult[(d >> 16) & 0xff]++;
    }
    if (e->next_mv_access.kind == 2) {
      uint32_t d = e->next_mv_access.ts - e->next_mv_access.prev_ts - 1;
      r->u16_mult[d & 0xffff]++;
      r->u8_mult[(d >> 16) & 0xff]++;
    }
    r->u8_mult[e->mv]++;
  }
  for (size_t i = 0; i < r->nalu; i++) {
    const or_alu_ev* e = &r->alu[i];
    uint8_t a = e->opcode == OP_ADD ? e->mv : e->next_mv;
    r->u8_mult[a]++;
    r->u8_mult[1]++;
    r->u8_mult[(uint8_t)(a + 1)]++;
  }
}

void or_record_free(or_record* r) {
  free(r->cpu); free(r->alu); free(r->jump); free(r->mi); free(r->io); free(r->mem);
  free(r->u8_mult); free(r->u16_mult); free(r->output);
  memset(r, 0, sizeof *r);
}

int or_chip_included(int chip, const or_record* r) {
  switch (chip) {
    case CHIP_CPU: return r->ncpu > 0;
    case CHIP_PROGRAM: return 1;
    case CHIP_ADDSUB: return r->nalu > 0;
    case CHIP_JUMP: return r->njump > 0;
    case CHIP_MEMORY: return r->nmem > 0;
    case CHIP_BYTE: return 1;
    case CHIP_MEMINSTRS: return r->nmi > 0;
    case CHIP_IO: return r->nio > 0;
  }
  return 0;
}

static size_t npot(size_t n) { size_t p = 1; while (p < n) p <<= 1; return p; }
static size_t npot16(size_t n) { size_t p = npot(n); return p < 16 ? 16 : p; }

static void word(fp* dst, uint32_t v) {
  for (int i = 0; i < 4; i++) dst[i] = (v >> (8 * i)) & 0xff;
}
/* KoalaBearWordRangeChecker::populate (operations/koala_bear_word.rs:29-45) */
static void word_rc(fp* dst, uint32_t v) {
  for (int i = 0; i < 8; i++) dst[i] = (v >> (i + 24)) & 1;
  dst[8] = dst[0] * dst[1];
  dst[9] = dst[8] * dst[2];
  dst[10] = dst[9] * dst[3];
  dst[11] = dst[10] * dst[4];
  dst[12] = dst[11] * dst[5];
  dst[13] = dst[12] * dst[6];
}

static void memacc_cols(fp* prev_value, fp* acc, const or_memacc* a) {
  /* MemoryReadWriteCols / MemoryWriteCols populate (memory/consistency/trace.rs:9-77) */
  *prev_value = a->kind == 2 ? a->prev_value : a->value;
  acc[0] = a->value;
  acc[1] = a->prev_ts;
  uint32_t d = a->ts - a->prev_ts - 1;
  acc[2] = d & 0xffff;
  acc[3] = (d >> 16) & 0xff;
}

size_t or_main_trace(int chip, const or_record* r, fp** out) {
  size_t h = 0, w = (size_t)OR_CHIPS[chip].main_w;
  fp* t = NULL;
  switch (chip) {
    case CHIP_CPU: { /* cpu/trace.rs:28-55,88-150; columns cpu/cols.rs:29-71 */
      h = npot(r->ncpu);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->ncpu; i++) {
        const or_cpu_ev* e = &r->cpu[i];
        fp* c = &t[i * w];
        int op = r->prog.ins[e->pc].opcode;
        c[0] = e->clk & 0xffff; c[1] = (e->clk >> 16) & 0xff;
        c[2] = e->pc; c[3] = e->next_pc;
        c[8] = (fp)op; word(&c[9], r->prog.ins[e->pc].op_a);
        c[4] = e->mp % OR_P; c[5] = e->next_mp % OR_P;
        c[6] = e->mv; c[7] = e->next_mv;
        c[14] = e->mv; c[19] = e->next_mv;
        if (e->mv_access.kind) { memacc_cols(&c[13], &c[14], &e->mv_access); c[23] = 1; }
        if (e->next_mv_access.kind == 2) { memacc_cols(&c[18], &c[19], &e->next_mv_access); c[24] = 1; }
        int is_alu = op == OP_ADD || op == OP_SUB;
        int is_jump = op == OP_LOOP_START || op == OP_LOOP_END;
        int is_mi = op == OP_FWD || op == OP_BWD;
        int is_io = op == OP_INPUT || op == OP_OUTPUT;
        c[25] = is_alu || is_jump || op == OP_OUTPUT;
        c[26] = is_alu; c[27] = is_jump; c[28] = is_io; c[29] = is_mi;
        c[30] = (fp)(is_alu + is_jump + is_mi + is_io);
      }
      break;
    }
    case CHIP_PROGRAM: { /* program/mod.rs:100-135 */
      h = npot16(r->prog.n);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->ncpu; i++) t[r->cpu[i].pc] = fp_add(t[r->cpu[i].pc], 1);
      break;
    }
    case CHIP_ADDSUB: { /* alu/mod.rs:63-146 */
      h = npot16(r->nalu);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->nalu; i++) {
        const or_alu_ev* e = &r->alu[i];
        fp* c = &t[i * w];
        uint8_t a = e->opcode == OP_ADD ? e->mv : e->next_mv;
        c[0] = e->pc;
        c[1] = (uint8_t)(a + 1);
        c[2] = ((unsigned)a + 1u > 255u) ? 1 : 0;
        c[3] = a; c[4] = 1;
        c[5] = e->opcode == OP_ADD; c[6] = e->opcode == OP_SUB;
      }
      break;
    }
    case CHIP_JUMP: { /* jump/trace.rs:32-97; cols jump/cols.rs:12-31 */
      h = npot16(r->njump);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->njump; i++) {
        const or_jump_ev* e = &r->jump[i];
        fp* c = &t[i * w];
        word(&c[0], e->pc); word_rc(&c[4], e->pc);
        word(&c[18], e->next_pc); word_rc(&c[22], e->next_pc);
        word(&c[36], e->dst);
        c[40] = e->mv;
        c[41] = e->mv ? fp_inv(e->mv) : 0;
        c[42] = e->mv ? 0 : 1;
        c[43] = e->opcode == OP_LOOP_START; c[44] = e->opcode == OP_LOOP_END;
      }
      break;
    }
    case CHIP_MEMORY: { /* memory/memory.rs:84-129 */
      h = npot16((r->nmem + 1) / 2);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->nmem; i++) {
        const or_mem_ev* e = &r->mem[i];
        fp* c = &t[(i / 2) * w + 6 * (i % 2)];
        c[0] = e->addr % OR_P; c[1] = e->init_ts; c[2] = e->final_ts;
        c[3] = e->init_v; c[4] = e->final_v; c[5] = 1;
      }
      break;
    }
    case CHIP_BYTE: { /* bytes/trace.rs:39-60 */
      h = 1 << 16;
      t = calloc(h * w, sizeof(fp));
      for (size_t v = 0; v < 256; v++) t[v * w + 0] = fp_from_u64(r->u8_mult[v]);
      for (size_t v = 0; v < 65536; v++) t[v * w + 1] = fp_from_u64(r->u16_mult[v]);
      break;
    }
    case CHIP_MEMINSTRS: { /* memory/instructions/trace.rs:30-97; cols cols.rs:13-35 */
      h = npot16(r->nmi);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->nmi; i++) {
        const or_meminstr_ev* e = &r->mi[i];
        fp* c = &t[i * w];
        c[0] = e->pc; c[1] = e->clk;
        word(&c[2], e->mp); word_rc(&c[6], e->mp);
        word(&c[20], e->next_mp); word_rc(&c[24], e->next_mp);
        c[38] = e->opcode == OP_FWD; c[39] = e->opcode == OP_BWD; c[40] = 1;
      }
      break;
    }
    case CHIP_IO: { /* io/mod.rs:72-121 */
      h = npot16(r->nio);
      t = calloc(h * w, sizeof(fp));
      for (size_t i = 0; i < r->nio; i++) {
        const or_io_ev* e = &r->io[i];
        fp* c = &t[i * w];
        c[0] = e->pc; c[1] = e->mp % OR_P; c[2] = e->mv;
        c[3] = e->opcode == OP_INPUT; c[4] = e->opcode == OP_OUTPUT;
      }
      break;
    }
  }
  *out = t;
  return h;
}

size_t or_prep_trace(int chip, const or_program* p, fp** out) {
  if (chip == CHIP_PROGRAM) { /* program/mod.rs:66-98 */
    size_t h = npot16(p->n);
    fp* t = calloc(h * 6, sizeof(fp));
    for (size_t i = 0; i < p->n; i++) {
      t[i * 6 + 0] = (fp)i;
      t[i * 6 + 1] = (fp)p->ins[i].opcode;
      word(&t[i * 6 + 2], p->ins[i].op_a);
    }
    *out = t;
    return h;
  }
  if (chip == CHIP_BYTE) { /* bytes/mod.rs:31-62: row (b,c) -> u8 = c, u16 = (b<<8)+c */
    size_t h = 1 << 16;
    fp* t = calloc(h * 2, sizeof(fp));
    for (size_t i = 0; i < h; i++) { t[2 * i] = i & 0xff; t[2 * i + 1] = (fp)i; }
    *out = t;
    return h;
  }
  *out = NULL;
  return 0;
}

/* ------------------------------------------------------------------ lookups */
enum { SRC_MAIN = 0, SRC_PREP = 1 };
enum { K_MEMORY = 1, K_PROGRAM = 2, K_ALU = 3, K_JUMP = 4, K_MEMINSTR = 5, K_IO = 6, K_BYTE = 7 };

static or_vcol vc_const(fp c) { or_vcol v; memset(&v, 0, sizeof v); v.c = c; return v; }
static or_vcol vc_col(int src, int col) {
  or_vcol v = vc_const(0); v.n = 1; v.src[0] = src; v.col[0] = col; v.w[0] = 1; return v;
}
static or_vcol vc_m(int col) { return vc_col(SRC_MAIN, col); }
static or_vcol vc_add_term(or_vcol v, int src, int col, fp w) {
  v.src[v.n] = src; v.col[v.n] = col; v.w[v.n] = w; v.n++; return v;
}
static or_vcol vc_word(int col) { /* Word::reduce: b0 + 2^8 b1 + 2^16 b2 + 2^24 b3 */
  or_vcol v = vc_const(0);
  for (int i = 0; i < 4; i++) v = vc_add_term(v, SRC_MAIN, col + i, 1u << (8 * i));
  return v;
}
static or_lookup lk(int kind, int nvals, const or_vcol* vals, or_vcol mult) {
  or_lookup l; memset(&l, 0, sizeof l);
  l.kind = kind; l.nvals = nvals;
  for (int i = 0; i < nvals; i++) l.vals[i] = vals[i];
  l.mult = mult;
  return l;
}

void or_chip_lookups_get(int chip, or_chip_lookups* o) {
  memset(o, 0, sizeof *o);
#define SEND(l) o->sends[o->nsends++] = (l)
#define RECV(l) o->recvs[o->nrecvs++] = (l)
  switch (chip) {
    case CHIP_CPU: { /* cpu/air.rs:28-98 -> air/program.rs, air/memory.rs, air/u8_air.rs */
      or_vcol clk = vc_add_term(vc_m(0), SRC_MAIN, 1, 1u << 16);
      or_vcol clk1 = clk; clk1.c = 1;
      or_vcol clk2 = clk; clk2.c = 2;
      { or_vcol v[7] = {vc_m(2), vc_m(8), vc_m(8), vc_m(9), vc_m(10), vc_m(11), vc_m(12)};
        SEND(lk(K_PROGRAM, 7, v, vc_m(30))); }
      { or_vcol v[4] = {vc_m(2), vc_m(8), vc_m(7), vc_m(6)}; SEND(lk(K_ALU, 4, v, vc_m(26))); }
      { or_vcol v[4] = {vc_m(2), vc_m(3), vc_m(8), vc_m(6)}; SEND(lk(K_JUMP, 4, v, vc_m(27))); }
      { or_vcol v[5] = {clk, vc_m(2), vc_m(8), vc_m(4), vc_m(5)}; SEND(lk(K_MEMINSTR, 5, v, vc_m(29))); }
      { or_vcol v[4] = {vc_m(2), vc_m(8), vc_m(4), vc_m(6)}; SEND(lk(K_IO, 4, v, vc_m(28))); }
      /* eval_memory_access(clk+1, mp, mv_access, mv_accessed) */
      { or_vcol v[3] = {vc_const(1), vc_const(0), vc_m(16)}; SEND(lk(K_BYTE, 3, v, vc_m(23))); }
      { or_vcol v[3] = {vc_const(0), vc_m(17), vc_const(0)}; SEND(lk(K_BYTE, 3, v, vc_m(23))); }
      { or_vcol v[3] = {vc_m(15), vc_m(4), vc_m(13)}; SEND(lk(K_MEMORY, 3, v, vc_m(23))); }
      { or_vcol v[3] = {clk1, vc_m(4), vc_m(14)}; RECV(lk(K_MEMORY, 3, v, vc_m(23))); }
      /* eval_memory_access(clk+2, mp, next_mv_access, next_mv_accessed) */
      { or_vcol v[3] = {vc_const(1), vc_const(0), vc_m(21)}; SEND(lk(K_BYTE, 3, v, vc_m(24))); }
      { or_vcol v[3] = {vc_const(0), vc_m(22), vc_const(0)}; SEND(lk(K_BYTE, 3, v, vc_m(24))); }
      { or_vcol v[3] = {vc_m(20), vc_m(4), vc_m(18)}; SEND(lk(K_MEMORY, 3, v, vc_m(24))); }
      { or_vcol v[3] = {clk2, vc_m(4), vc_m(19)}; RECV(lk(K_MEMORY, 3, v, vc_m(24))); }
      /* range_check_u8(mv, is_real) */
      { or_vcol v[3] = {vc_const(0), vc_m(6), vc_const(0)}; SEND(lk(K_BYTE, 3, v, vc_m(30))); }
      /* eval_clk -> eval_range_check_24bits(clk, clk16, clk8, is_real) */
      { or_vcol v[3] = {vc_const(1), vc_const(0), vc_m(0)}; SEND(lk(K_BYTE, 3, v, vc_m(30))); }
      { or_vcol v[3] = {vc_const(0), vc_m(1), vc_const(0)}; SEND(lk(K_BYTE, 3, v, vc_m(30))); }
      break;
    }
    case CHIP_PROGRAM: { /* program/mod.rs:150-163 */
      or_vcol v[7] = {vc_col(SRC_PREP, 0), vc_col(SRC_PREP, 1), vc_col(SRC_PREP, 1),
                      vc_col(SRC_PREP, 2), vc_col(SRC_PREP, 3), vc_col(SRC_PREP, 4),
                      vc_col(SRC_PREP, 5)};
      RECV(lk(K_PROGRAM, 7, v, vc_m(0)));
      break;
    }
    case CHIP_ADDSUB: { /* alu/mod.rs:155-193, operations/add.rs:44-76 */
      or_vcol is_real = vc_add_term(vc_m(5), SRC_MAIN, 6, 1);
      { or_vcol v[3] = {vc_const(0), vc_m(3), vc_const(0)}; SEND(lk(K_BYTE, 3, v, is_real)); }
      { or_vcol v[3] = {vc_const(0), vc_m(4), vc_const(0)}; SEND(lk(K_BYTE, 3, v, is_real)); }
      { or_vcol v[3] = {vc_const(0), vc_m(1), vc_const(0)}; SEND(lk(K_BYTE, 3, v, is_real)); }
      { or_vcol v[4] = {vc_m(0), vc_const(OP_ADD), vc_m(1), vc_m(3)}; RECV(lk(K_ALU, 4, v, vc_m(5))); }
      { or_vcol v[4] = {vc_m(0), vc_const(OP_SUB), vc_m(3), vc_m(1)}; RECV(lk(K_ALU, 4, v, vc_m(6))); }
      break;
    }
    case CHIP_JUMP: { /* jump/air.rs:72-81 */
      or_vcol op = vc_const(0);
      op = vc_add_term(op, SRC_MAIN, 43, OP_LOOP_START);
      op = vc_add_term(op, SRC_MAIN, 44, OP_LOOP_END);
      or_vcol v[4] = {vc_word(0), vc_word(18), op, vc_m(40)};
      RECV(lk(K_JUMP, 4, v, vc_add_term(vc_m(43), SRC_MAIN, 44, 1)));
      break;
    }
    case CHIP_MEMORY: { /* memory/memory.rs:131-146 */
      for (int e = 0; e < 2; e++) {
        int b = 6 * e;
        { or_vcol v[3] = {vc_m(b + 1), vc_m(b + 0), vc_m(b + 3)}; RECV(lk(K_MEMORY, 3, v, vc_m(b + 5))); }
        { or_vcol v[3] = {vc_m(b + 2), vc_m(b + 0), vc_m(b + 4)}; SEND(lk(K_MEMORY, 3, v, vc_m(b + 5))); }
      }
      break;
    }
    case CHIP_BYTE: { /* bytes/air.rs:21-44 */
      { or_vcol v[3] = {vc_const(0), vc_col(SRC_PREP, 0), vc_const(0)}; RECV(lk(K_BYTE, 3, v, vc_m(0))); }
      { or_vcol v[3] = {vc_const(1), vc_const(0), vc_col(SRC_PREP, 1)}; RECV(lk(K_BYTE, 3, v, vc_m(1))); }
      break;
    }
    case CHIP_MEMINSTRS: { /* memory/instructions/air.rs:65-75 */
      or_vcol op = vc_const(0);
      op = vc_add_term(op, SRC_MAIN, 38, OP_FWD);
      op = vc_add_term(op, SRC_MAIN, 39, OP_BWD);
      or_vcol v[5] = {vc_m(1), vc_m(0), op, vc_word(2), vc_word(20)};
      RECV(lk(K_MEMINSTR, 5, v, vc_add_term(vc_m(38), SRC_MAIN, 39, 1)));
      break;
    }
    case CHIP_IO: { /* io/mod.rs:127-141 */
      or_vcol op = vc_const(0);
      op = vc_add_term(op, SRC_MAIN, 3, OP_INPUT);
      op = vc_add_term(op, SRC_MAIN, 4, OP_OUTPUT);
      or_vcol v[4] = {vc_m(0), op, vc_m(1), vc_m(2)};
      RECV(lk(K_IO, 4, v, vc_add_term(vc_m(3), SRC_MAIN, 4, 1)));
      break;
    }
  }
#undef SEND
#undef RECV
}

int or_perm_width(int chip) {
  or_chip_lookups l;
  or_chip_lookups_get(chip, &l);
  int n = l.nsends + l.nrecvs;
  return n ? (n + 1) / 2 + 1 : 0;
}

/* ------------------------------------------------------------ AIR constraints */
static inline ef E(fp x) { return ef_from_fp(x); }
static inline ef A(ef a, ef b) { return ef_add(a, b); }
static inline ef S(ef a, ef b) { return ef_sub(a, b); }
static inline ef M(ef a, ef b) { return ef_mul(a, b); }
static inline void emit(or_folder* f, ef c) { f->acc = ef_add(ef_mul(f->acc, f->alpha), c); }
static inline ef boolc(ef x) { return M(x, S(x, E(1))); } /* assert_bool: x*(x-1) */

#define L(i) (f->main_l[i])
#define N(i) (f->main_n[i])

static ef reduce_word(const ef* w) {
  ef r = w[0];
  r = A(r, M(w[1], E(1u << 8)));
  r = A(r, M(w[2], E(1u << 16)));
  r = A(r, M(w[3], E(1u << 24)));
  return r;
}

/* KoalaBearWordRangeChecker::range_check (operations/koala_bear_word.rs:47-106) */
static void word_range_check(or_folder* f, const ef* v, const ef* rc, ef is_real) {
  ef recomposed = E(0);
  for (int i = 0; i < 8; i++) {
    emit(f, M(is_real, boolc(rc[i])));
    recomposed = A(recomposed, M(E(1u << i), rc[i]));
  }
  emit(f, M(is_real, S(recomposed, v[3])));
  emit(f, M(is_real, rc[7]));
  emit(f, M(is_real, S(rc[8], M(rc[0], rc[1]))));
  emit(f, M(is_real, S(rc[9], M(rc[8], rc[2]))));
  emit(f, M(is_real, S(rc[10], M(rc[9], rc[3]))));
  emit(f, M(is_real, S(rc[11], M(rc[10], rc[4]))));
  emit(f, M(is_real, S(rc[12], M(rc[11], rc[5]))));
  emit(f, M(is_real, S(rc[13], M(rc[12], rc[6]))));
  emit(f, M(M(is_real, rc[13]), A(A(v[0], v[1]), v[2])));
}

static void eval_cpu(or_folder* f) { /* cpu/air.rs:28-186 */
  ef c65536 = E(1u << 16);
  ef clk = A(M(c65536, L(1)), L(0));
  /* eval_registers -> eval_memory_access(clk+1, mp, mv_access, mv_accessed) */
  emit(f, boolc(L(23)));
  { ef diff = S(S(A(clk, E(1)), L(15)), E(1));
    emit(f, M(L(23), S(diff, A(L(16), M(L(17), c65536))))); }
  /* eval_memory_access(clk+2, mp, next_mv_access, next_mv_accessed) */
  emit(f, boolc(L(24)));
  { ef diff = S(S(A(clk, E(2)), L(20)), E(1));
    emit(f, M(L(24), S(diff, A(L(21), M(L(22), c65536))))); }
  /* when(is_mv_immutable).assert_eq(mv_val, mv_access.prev_value) */
  emit(f, M(L(25), S(L(14), L(13))));
  /* eval_clk */
  emit(f, M(f->is_first, clk));
  { ef next_clk = A(M(c65536, N(1)), N(0));
    emit(f, M(M(f->is_trans, N(30)), S(A(clk, E(2)), next_clk))); }
  emit(f, M(L(30), S(clk, A(L(0), M(L(1), c65536)))));
  /* eval_pc */
  emit(f, M(M(f->is_trans, N(30)), S(L(3), N(2))));
  emit(f, M(M(M(f->is_trans, L(30)), S(L(27), E(1))), S(L(3), A(L(2), E(1)))));
  /* eval_is_real */
  emit(f, boolc(L(30)));
  emit(f, M(f->is_first, S(L(30), E(1))));
  emit(f, M(M(f->is_trans, S(L(30), E(1))), N(30)));
  /* booleans */
  emit(f, boolc(L(26)));
  emit(f, boolc(L(27)));
  emit(f, boolc(L(29)));
  emit(f, boolc(L(28)));
  emit(f, boolc(L(25)));
  emit(f, boolc(L(23)));
  emit(f, boolc(L(24)));
}

static void eval_addsub(or_folder* f) { /* alu/mod.rs:155-193, operations/add.rs:44-76 */
  ef is_real = A(L(5), L(6));
  emit(f, boolc(L(5)));
  emit(f, boolc(L(6)));
  emit(f, boolc(is_real));
  ef base = E(256);
  ef overflow = S(A(L(3), L(4)), L(1));
  emit(f, M(is_real, M(overflow, S(overflow, base))));
  emit(f, M(is_real, M(L(2), S(overflow, base))));
  emit(f, M(is_real, M(S(L(2), E(1)), overflow)));
  emit(f, M(is_real, boolc(L(2))));
  emit(f, M(is_real, boolc(is_real)));
}

static void eval_jump(or_folder* f) { /* jump/air.rs:22-82, operations/is_zero.rs:48-66 */
  ef is_real = A(L(43), L(44));
  emit(f, boolc(L(43)));
  emit(f, boolc(L(44)));
  emit(f, boolc(is_real));
  ef is_zero = S(E(1), M(L(41), L(40)));
  emit(f, M(is_real, S(is_zero, L(42))));
  emit(f, M(is_real, boolc(L(42))));
  emit(f, M(M(is_real, L(42)), L(40)));
  ef npc = reduce_word(&L(18)), dst = reduce_word(&L(36)), pc = reduce_word(&L(0));
  emit(f, M(M(L(43), L(42)), S(npc, dst)));
  emit(f, M(M(L(43), S(L(42), E(1))), S(npc, A(pc, E(1)))));
  emit(f, M(M(L(44), S(L(42), E(1))), S(npc, dst)));
  emit(f, M(M(L(44), L(42)), S(npc, A(pc, E(1)))));
  word_range_check(f, &L(0), &L(4), is_real);
  word_range_check(f, &L(18), &L(22), is_real);
}

static void eval_meminstrs(or_folder* f) { /* memory/instructions/air.rs:25-76 */
  ef is_real = A(L(38), L(39));
  emit(f, boolc(L(38)));
  emit(f, boolc(L(39)));
  emit(f, boolc(is_real));
  ef mp = reduce_word(&L(2)), nmp = reduce_word(&L(20));
  emit(f, M(L(38), S(nmp, A(mp, E(1)))));
  emit(f, M(L(39), S(nmp, S(mp, E(1)))));
  emit(f, M(M(f->is_trans, N(40)), S(nmp, reduce_word(&N(2)))));
  word_range_check(f, &L(2), &L(6), L(40));
  word_range_check(f, &L(20), &L(24), L(40));
}

static void eval_io(or_folder* f) { /* io/mod.rs:127-141 */
  emit(f, boolc(L(3)));
  emit(f, boolc(L(4)));
  emit(f, boolc(A(L(3), L(4))));
}

static ef vcol_eval(const or_vcol* v, const ef* prep, const ef* main) {
  ef r = E(v->c);
  for (int i = 0; i < v->n; i++)
    r = A(r, M(E(v->w[i]), v->src[i] == SRC_PREP ? prep[v->col[i]] : main[v->col[i]]));
  return r;
}

/* eval_permutation_constraints (crates/stark/src/permutation.rs:157-272) */
static void eval_perm(int chip, or_folder* f) {
  or_chip_lookups lu;
  or_chip_lookups_get(chip, &lu);
  int nint = lu.nsends + lu.nrecvs;
  int pw = nint ? (nint + 1) / 2 + 1 : 0;
  if (!pw) return;
  const or_lookup* all[32];
  int is_send[32];
  for (int i = 0; i < lu.nsends; i++) { all[i] = &lu.sends[i]; is_send[i] = 1; }
  for (int i = 0; i < lu.nrecvs; i++) { all[lu.nsends + i] = &lu.recvs[i]; is_send[lu.nsends + i] = 0; }
  for (int b = 0; b < pw - 1; b++) {
    ef rlcs[2], ms[2];
    int cnt = 0;
    for (int j = 2 * b; j < 2 * b + 2 && j < nint; j++) {
      const or_lookup* l = all[j];
      ef rlc = f->perm_alpha;
      ef bp = E(1);
      rlc = A(rlc, M(bp, E((fp)l->kind)));
      for (int k = 0; k < l->nvals; k++) {
        bp = M(bp, f->perm_beta);
        rlc = A(rlc, M(bp, vcol_eval(&l->vals[k], f->prep_l, f->main_l)));
      }
      rlcs[cnt] = rlc;
      ef m = vcol_eval(&l->mult, f->prep_l, f->main_l);
      ms[cnt] = is_send[j] ? m : ef_neg(m);
      cnt++;
    }
    ef product = E(1), numerator = E(0);
    for (int i = 0; i < cnt; i++) {
      product = M(product, rlcs[i]);
      ef abc = E(1);
      for (int j = 0; j < cnt; j++) if (j != i) abc = M(abc, rlcs[j]);
      numerator = A(numerator, M(ms[i], abc));
    }
    emit(f, S(M(product, f->perm_l[b]), numerator));
  }
  ef sum_l = E(0), sum_n = E(0);
  for (int b = 0; b < pw - 1; b++) { sum_l = A(sum_l, f->perm_l[b]); sum_n = A(sum_n, f->perm_n[b]); }
  ef phi_l = f->perm_l[pw - 1], phi_n = f->perm_n[pw - 1];
  emit(f, M(f->is_first, S(phi_l, sum_l)));
  emit(f, M(f->is_trans, S(S(phi_n, phi_l), sum_n)));
  emit(f, M(f->is_last, S(phi_l, f->cumsum)));
}

void or_eval_chip(int chip, or_folder* f) { /* Chip::eval (crates/stark/src/chip.rs:222-228) */
  switch (chip) {
    case CHIP_CPU: eval_cpu(f); break;
    case CHIP_ADDSUB: eval_addsub(f); break;
    case CHIP_JUMP: eval_jump(f); break;
    case CHIP_MEMINSTRS: eval_meminstrs(f); break;
    case CHIP_IO: eval_io(f); break;
    default: break; /* Program, Memory, Byte: lookups only */
  }
  eval_perm(chip, f);
}
