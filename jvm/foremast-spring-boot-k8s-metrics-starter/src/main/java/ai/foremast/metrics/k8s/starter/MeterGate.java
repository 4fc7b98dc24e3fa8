package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.Meter;
import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.config.MeterFilter;
import io.micrometer.core.instrument.config.MeterFilterReply;

import java.util.Arrays;
import java.util.Collections;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.concurrent.ConcurrentHashMap;
import java.util.stream.Collectors;

/**
 * The common-metrics gate: with {@code k8s.metrics.enable-common-metrics-filter}
 * a meter is exposed only if (in this order) its {@code management.metrics.enable.*}
 * entry (dotted-prefix lookup, then {@code all}) says so, it is whitelisted,
 * it is not blacklisted and it carries a configured prefix or tag value.
 * Whitelist / blacklist change at runtime through {@link K8sMetricsEndpoint}.
 * Semantics mirror {@code foremast_amd/emitter/metrics.py:CommonMetricsFilter}
 * (and the reference starter's CommonMetricsFilter.java:38-196).
 */
public class MeterGate implements MeterFilter {

    private final K8sMetricsProperties props;
    private final Map<String, Boolean> enable;
    private final Set<String> whitelist = ConcurrentHashMap.newKeySet();
    private final Set<String> blacklist = ConcurrentHashMap.newKeySet();
    private final List<String> prefixes;
    private final Map<String, String> tagRules = new LinkedHashMap<>();

    public MeterGate(K8sMetricsProperties props, Map<String, Boolean> enable) {
        this.props = props;
        this.enable = enable == null ? Collections.emptyMap() : enable;
        tokens(props.getCommonMetricsWhitelist()).forEach(t -> whitelist.add(meterName(t)));
        tokens(props.getCommonMetricsBlacklist()).forEach(t -> blacklist.add(meterName(t)));
        prefixes = tokens(props.getCommonMetricsPrefix());
        for (String rule : tokens(props.getCommonMetricsTagRules())) {
            String[] kv = rule.split(":");
            if (kv.length != 2) {
                throw new IllegalArgumentException("Invalid common tag name value pair:" + rule);
            }
            tagRules.put(kv[0].trim(), kv[1].trim());
        }
    }

    static List<String> tokens(String csv) {
        if (csv == null || csv.trim().isEmpty()) {
            return Collections.emptyList();
        }
        return Arrays.stream(csv.split(",")).map(String::trim).filter(s -> !s.isEmpty())
                .collect(Collectors.toList());
    }

    /** Prometheus family name to Micrometer meter name: '_' to '.', unit suffix dropped. */
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
        String n = name;
        while (!n.isEmpty()) {
            Boolean v = enable.get(n);
            if (v != null) {
                return v;
            }
            int dot = n.lastIndexOf('.');
            n = dot < 0 ? "" : n.substring(0, dot);
        }
        return enable.get("all");
    }

    @Override
    public MeterFilterReply accept(Meter.Id id) {
        if (!props.isEnableCommonMetricsFilter()) {
            return MeterFilterReply.NEUTRAL;
        }
        String name = id.getName();
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
        for (Tag t : id.getTags()) {
            String want = tagRules.get(t.getKey());
            if (want != null && want.equals(t.getValue())) {
                return MeterFilterReply.ACCEPT;
            }
        }
        return MeterFilterReply.DENY;
    }

    public boolean enableMetric(String name) {
        if (!props.isEnableCommonMetricsFilterAction()) {
            return false;
        }
        String n = meterName(name);
        blacklist.remove(n);
        whitelist.add(n);
        return true;
    }

    public boolean disableMetric(String name) {
        if (!props.isEnableCommonMetricsFilterAction()) {
            return false;
        }
        String n = meterName(name);
        whitelist.remove(n);
        blacklist.add(n);
        return true;
    }
}
