/* qjson.h - minimal JSON DOM (objects, arrays, strings, numbers, literals)
 * for config.json and safetensors headers. */
#ifndef QJSON_H
#define QJSON_H

#include <stddef.h>

typedef enum { QJ_NULL, QJ_BOOL, QJ_NUM, QJ_STR, QJ_ARR, QJ_OBJ } qj_type_t;

typedef struct qj {
    qj_type_t type;
    double num;
    char *str;            /* QJ_STR value */
    char **keys;          /* QJ_OBJ member names */
    struct qj **items;    /* QJ_ARR elements / QJ_OBJ values */
    int n;
} qj_t;

qj_t *qj_parse(const char *text, size_t len);   /* NULL on syntax error */
void qj_free(qj_t *v);
const qj_t *qj_get(const qj_t *obj, const char *key);
/* dotted path lookup: "talker_config.code_predictor_config.hidden_size" */
const qj_t *qj_path(const qj_t *root, const char *path);
int qj_int(const qj_t *root, const char *path, int def);
float qj_float(const qj_t *root, const char *path, float def);
/* reads up to max ints of an array; returns the count read */
int qj_ints(const qj_t *root, const char *path, int *out, int max);
char *qj_read_file(const char *path, size_t *len);

#endif
