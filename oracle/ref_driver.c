/* ref_driver.c -- loops over the reference's own bloom_filter.c strategy functions
 * (src/bloom_filter.h:43-69), linked with the unmodified reference sources into
 * _ref/libbloomref.so. TEST INFRASTRUCTURE ONLY. */
#include <stdint.h>

#include "bloom_filter.h"

void ref_add_all(bloom_filter_strategy_t * s, const int32_t * keys, uint64_t n)
{
    for (uint64_t i = 0; i < n; i++) s->add(s->filter, keys[i]);
}

uint64_t ref_count(bloom_filter_strategy_t * s, const int32_t * keys, uint64_t n)
{
    uint64_t c = 0;
    for (uint64_t i = 0; i < n; i++) c += s->contains(s->filter, keys[i]) ? 1 : 0;
    return c;
}
