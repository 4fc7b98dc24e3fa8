package ai.foremast.metrics.servlet;

import io.micrometer.core.instrument.Meter;
import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.config.MeterFilter;
import io.micrometer.core.instrument.config.MeterFilterReply;

import java.util.ArrayList;
import java.util.Collections;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.concurrent.ConcurrentHashMap;

/**
 * The common-metrics filter of the servlet module (the reference 4.x / 1.x
 * starters' role: foremast-spring-4x-k8s-metrics/.../CommonMetricsFilter.java),
 * configured from plain settings (init parameters, system properties) instead
 * of Spring properties, Java 8 only.
 *
 * <p>With {@code enableCommonMetricsFilter=true} a meter is exposed when, in
 * this order: an {@code enable.<dotted prefix>} / {@code enable.all} setting
 * says so, it is whitelisted (NEUTRAL), it is not blacklisted (DENY), its name
 * starts with a configured prefix (ACCEPT), or it carries a configured
 * {@code tag:value} (ACCEPT); anything else is denied.  With
 * {@code enableCommonMetricsFilterAction=true} {@link #enableMetric} /
 * {@link #disableMetric} move a metric between the lists at runtime
 * ({@link MetricsControlServlet}).  Names are Micrometer meter names; a
 * Prometheus family name ({@code jvm_memory_used_bytes}) is accepted too.
 *
 * <p>The decisions are pinned by {@code src/test/resources/gate-vectors.txt},
 * the same table {@code tests/test_jvm_starter.py} runs through the Python
 * emitter's filter ({@code foremast_amd/emitter/metrics.py}).
 */
public class CommonMetricsGate implements MeterFilter {

    private final boolean enabled;
    private final boolean actions;
    private final Map<String, Boolean> enable = new LinkedHashMap<>();
    private final Set<String> whitelist = ConcurrentHashMap.newKeySet();
    private final Set<String> blacklist = ConcurrentHashMap.newKeySet();
    private final List<String> prefixes;
    private final Map<String, String> tagRules = new LinkedHashMap<>();

    public CommonMetricsGate(Map<String, String> settings) {
        enabled = "true".equalsIgnoreCase(settings.get("enableCommonMetricsFilter"));
        actions = "true".equalsIgnoreCase(settings.get("enableCommonMetricsFilterAction"));
        for (String t : tokens(settings.get("commonMetricsWhitelist"))) {
            whitelist.add(meterName(t));
        }
        for (String t : tokens(settings.get("commonMetricsBlacklist"))) {
            blacklist.add(meterName(t));
        }
        prefixes = tokens(settings.get("commonMetricsPrefix"));
        for (String rule : tokens(settings.get("commonMetricsTagRules"))) {
            String[] kv = rule.split(":");
            if (kv.length != 2) {
                throw new IllegalArgumentException("Invalid common tag name value pair:" + rule);
            }
            tagRules.put(kv[0].trim(), kv[1].trim());
        }
        for (Map.Entry<String, String> e : settings.entrySet()) {
            if (e.getKey().startsWith("enable.")) {
                enable.put(e.getKey().substring("enable.".length()), "true".equalsIgnoreCase(e.getValue().trim()));
            }
        }
    }

    static List<String> tokens(String csv) {
        if (csv == null || csv.trim().isEmpty()) {
            return Collections.emptyList();
        }
        List<String> out = new ArrayList<>();
        for (String s : csv.split(",")) {
            if (!s.trim().isEmpty()) {
                out.add(s.trim());
            }
        }
        return out;
    }

    /** Prometheus family name to meter name: unit suffix dropped, '_' to '.'. */
    static String meterName(String name) {
        String n = name;
        for (String suffix : new String[] {"_seconds_max", "_seconds", "_bytes", "_total", "_max"}) {
            if (n.endsWith(suffix)) {
                n = n.substring(0, n.length() - suffix.length());
                break;
            }
        }
        return n.replace('_', '.');
    }

    private Boolean lookupEnable(String name) {
        if (enable.isEmpty()) {
            return null;
        }
        for (String n = name; !n.isEmpty(); ) {
            Boolean v = enable.get(n);
            if (v != null) {
                return v;
            }
            int dot = n.lastIndexOf('.');
            n = dot < 0 ? "" : n.substring(0, dot);
        }
        return enable.get("all");
    }

    /** The decision for a meter name and its tags (what {@link #accept} applies). */
    public MeterFilterReply decide(String name, Iterable<Tag> tags) {
        if (!enabled) {
            return MeterFilterReply.NEUTRAL;
        }
        Boolean en = lookupEnable(name);
        if (en != null) {
            return en ? MeterFilterReply.NEUTRAL : MeterFilterReply.DENY;
        }
        if (whitelist.contains(name)) {
            return MeterFilterReply.NEUTRAL;
        }
        if (blacklist.contains(name)) {
            return MeterFilterReply.DENY;
        }
        for (String p : prefixes) {
            if (name.startsWith(p)) {
                return MeterFilterReply.ACCEPT;
            }
        }
        for (Tag t : tags) {
            String want = tagRules.get(t.getKey());
            if (want != null && want.equals(t.getValue())) {
                return MeterFilterReply.ACCEPT;
            }
        }
        return MeterFilterReply.DENY;
    }

    @Override
    public MeterFilterReply accept(Meter.Id id) {
        return decide(id.getName(), id.getTags());
    }

    /** Runtime whitelist (false when runtime actions are off). */
    public boolean enableMetric(String name) {
        if (!actions) {
            return false;
        }
        String n = meterName(name);
        blacklist.remove(n);
        whitelist.add(n);
        return true;
    }

    /** Runtime blacklist (false when runtime actions are off). */
    public boolean disableMetric(String name) {
        if (!actions) {
            return false;
        }
        String n = meterName(name);
        whitelist.remove(n);
        blacklist.add(n);
        return true;
    }
}
