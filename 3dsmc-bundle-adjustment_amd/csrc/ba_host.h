// ba_host.h — internal host-side helpers shared by the libmiba translation units.
#pragma once
#include <string>

#include "../../include/ba.h"

// Sets the context-free error text returned by ba_last_error(NULL).
void miba_set_error(const std::string& msg);
// MIBA_DUMP_DIR window capture (ba_io.cpp); no-op when the variable is unset.
void miba_maybe_dump_window(const ba_problem* p, const ba_options* o);
