#!/usr/bin/env python3
"""Makes _app/list_batched.c: the reference's list.c with INTEGRATION.md's batch integration applied
(TEST INFRASTRUCTURE ONLY; the C1 test `test_reference_app_batched_run` runs the result):

  * list__compressor_start (src/list.c:1047-1063): the grabbed victims go to ONE
    tyche_buffers_compress call instead of one buffer__compress each; per victim the status and the
    list__update install are the unchanged code's, and any failure keeps the page raw;
  * the list__search restore (src/list.c:572): buffer__decompress -> tyche_buffer_restore, so
    concurrent hits share GPU launches through the engine's restore queue;
  * list__initialize (src/list.c:169): the queue is started once, next to the compressor pool.

Every edit is anchored on the reference text and must match exactly once, so a different list.c
fails the build instead of producing something else.
    python3 patch_batched.py <reference list.c> <output>
"""
import sys

EDITS = [
    # 1: prototypes of the engine's batch calls (include/tyche_codec.h)
    ('#include "list.h"\n',
     '#include "list.h"\n'
     '/* INTEGRATION.md: the engine\'s batch calls (include/tyche_codec.h) */\n'
     'int tyche_buffers_compress(Buffer **bufs, void **compressed, int *status, size_t n, int compressor_id,\n'
     '                           int compressor_level);\n'
     'int tyche_restore_queue_start(int max_batch, int max_wait_us);\n'
     'int tyche_buffer_restore(Buffer *buf, int compressor_id);\n'),
    # 2: the compressor pool's per-victim loop -> one batch
    ('    for(int i = 0; i < work_me_count; i++) {\n'
     '      // Compress the buffer\'s data.  Lean on list__update() for the heavy lifting and CoW work.\n'
     '      if(work_me[i]->flags & compressed)\n'
     '        continue;\n'
     '      rv = buffer__compress(work_me[i], &compressed_data, comp->compressor_id, comp->compressor_level);\n'
     '      if(rv == E_BUFFER_ALREADY_COMPRESSED)\n'
     '        continue;\n',
     '    /* INTEGRATION.md: one GPU batch per grabbed set of victims (was one buffer__compress each) */\n'
     '    void *batch_out[COMPRESSOR_BATCH_SIZE];\n'
     '    int batch_st[COMPRESSOR_BATCH_SIZE];\n'
     '    Buffer *batch_bufs[COMPRESSOR_BATCH_SIZE];\n'
     '    int batch_n = 0;\n'
     '    for(int i = 0; i < work_me_count; i++)\n'
     '      if(!(work_me[i]->flags & compressed))\n'
     '        batch_bufs[batch_n++] = work_me[i];\n'
     '    if(batch_n > 0) {\n'
     '      int batch_rv = tyche_buffers_compress(batch_bufs, batch_out, batch_st, (size_t)batch_n, comp->compressor_id,\n'
     '                                            comp->compressor_level);\n'
     '      if(batch_rv != E_OK)\n'
     '        for(int i = 0; i < batch_n; i++)\n'
     '          batch_st[i] = batch_rv;\n'
     '    }\n'
     '    for(int i = 0; i < batch_n; i++) {\n'
     '      work_me[i] = batch_bufs[i];\n'
     '      compressed_data = batch_out[i];\n'
     '      rv = batch_st[i];\n'
     '      if(rv != E_OK)   /* already compressed, or a failure: the page stays raw */\n'
     '        continue;\n'),
    # 3: the restore site
    ('      decompress_rv = buffer__decompress(*buf, list->compressor_id);\n',
     '      decompress_rv = tyche_buffer_restore(*buf, list->compressor_id);   /* INTEGRATION.md: restore queue */\n'),
    # 4: start the queue once, next to the compressor pool
    ('  (*list)->compressor_count = compressor_count;\n',
     '  (*list)->compressor_count = compressor_count;\n'
     '  tyche_restore_queue_start(1024, 50);   /* INTEGRATION.md: restore queue, once */\n'),
]


def main():
    src, dst = sys.argv[1], sys.argv[2]
    text = open(src).read()
    for old, new in EDITS:
        n = text.count(old)
        if n != 1:
            raise SystemExit(f"patch_batched: anchor found {n} times (want 1):\n{old}")
        text = text.replace(old, new)
    open(dst, "w").write(text)


if __name__ == "__main__":
    main()
