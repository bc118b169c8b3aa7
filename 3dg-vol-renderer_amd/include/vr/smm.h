// Reference header name (include/smm.h) mapped onto the MI355X host API.
#pragma once
#include "vol_renderer.h"
