extern "C" const char* rtw_build_id(void) { return "e8cbf99f0526a8a3"; }
