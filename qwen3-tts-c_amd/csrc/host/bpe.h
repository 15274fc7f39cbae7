/* bpe.h - Qwen2 byte-level BPE text tokenizer over a model directory's
 * vocab.json / merges.txt / tokenizer_config.json (host C11; bpe.c). */
#ifndef QTTS_BPE_H
#define QTTS_BPE_H

typedef struct qtok qtok_t;

qtok_t *qtok_load(const char *model_dir);   /* NULL (message on stderr) on failure */
void qtok_free(qtok_t *t);
/* text (UTF-8, NFC) -> malloc'd ids (caller frees); returns the count, -1 on error */
int qtok_encode(const qtok_t *t, const char *text, int **ids);

#endif
